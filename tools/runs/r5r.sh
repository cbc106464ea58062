# round 5, run R: the first tier with its dictionary staging loads batched (one wait per 16 steps
# instead of one per table step): C3 at 32/64/128 blocks per CU, C2 at 2^30 (the headline), the rest at 2^28
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r5r_rates.jsonl
rate() {  # workload engine candidates tag [env...]
  local w=$1 e=$2 n=$3 tag=$4; shift 4
  env "$@" timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5r_b.json 2> gpurun_out/r5r_b.err || { tail -20 gpurun_out/r5r_b.err; return 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/r5r_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'n': $n, 'tag': '$tag', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5r_rates.jsonl
}
for sb in 1 16; do
  for b in 32 64; do rate bectoken_batch_overflow asm 268435456 sb${sb}_bpc$b MYTHGPU_JIT_BPC=$b MYTHGPU_JIT_ASM_STAGE_BATCH=$sb || exit 1; done
  rate token_transfer_underflow asm 1073741824 sb$sb MYTHGPU_JIT_ASM_STAGE_BATCH=$sb || exit 1
  for w in suicide_kill walletlibrary_kill etherstore_reentrancy; do rate $w asm 268435456 sb$sb MYTHGPU_JIT_ASM_STAGE_BATCH=$sb || exit 1; done
done
cat gpurun_out/r5r_rates.jsonl
