# round 5, run M: blocks per CU for the first tier's search kernels (C1, C3, C4 at 2^28), against the
# O3 kernel: where the first tier trails O3 with about the same instructions per candidate
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r5m_rates.jsonl
rate() {  # workload engine candidates tag [env...]
  local w=$1 e=$2 n=$3 tag=$4; shift 4
  env "$@" timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5m_b.json 2> gpurun_out/r5m_b.err || { tail -20 gpurun_out/r5m_b.err; return 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/r5m_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'tag': '$tag', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5m_rates.jsonl
}
for w in bectoken_batch_overflow suicide_kill walletlibrary_kill; do
  rate $w jit 268435456 o3 || exit 1
  for b in 16 32 64 128; do rate $w asm 268435456 bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
done
cat gpurun_out/r5m_rates.jsonl
