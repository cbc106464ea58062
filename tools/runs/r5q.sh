# round 5, run Q: blocks per CU for the first tier's search kernels (C3's first tier ran 283 -> 424 G/s
# at 64 -> 32 blocks per CU in run P): C2 at the headline's 2^30 and at 2^28, C1, C4, etherstore
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r5q_rates.jsonl
rate() {  # workload engine candidates tag [env...]
  local w=$1 e=$2 n=$3 tag=$4; shift 4
  env "$@" timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5q_b.json 2> gpurun_out/r5q_b.err || { tail -20 gpurun_out/r5q_b.err; return 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/r5q_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'n': $n, 'tag': '$tag', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5q_rates.jsonl
}
for b in 16 32 64 128; do rate token_transfer_underflow asm 1073741824 bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
for b in 8 16 32; do rate token_transfer_underflow asm 268435456 bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
for w in suicide_kill walletlibrary_kill etherstore_reentrancy bectoken_batch_overflow; do
  for b in 8 16 32; do rate $w asm 268435456 bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
done
for b in 32 64; do rate token_transfer_underflow jit 1073741824 o3_bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
cat gpurun_out/r5q_rates.jsonl
