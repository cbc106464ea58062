# round 5, run S: the first tier's end-of-wave atomicMin skipped when the hit word is already lower
# (MYTHGPU_JIT_ASM_EXIT_SKIP=1) against the default, C3 at 64 and 32 blocks per CU, C2 at 2^30, C1/C4 at 2^28
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r5s_rates.jsonl
rate() {  # workload engine candidates tag [env...]
  local w=$1 e=$2 n=$3 tag=$4; shift 4
  env "$@" timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5s_b.json 2> gpurun_out/r5s_b.err || { tail -20 gpurun_out/r5s_b.err; return 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/r5s_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'n': $n, 'tag': '$tag', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5s_rates.jsonl
}
for x in 0 1; do
  rate bectoken_batch_overflow asm 268435456 skip${x}_bpc64 MYTHGPU_JIT_ASM_EXIT_SKIP=$x || exit 1
  rate bectoken_batch_overflow asm 268435456 skip${x}_bpc32 MYTHGPU_JIT_ASM_EXIT_SKIP=$x MYTHGPU_JIT_BPC=32 || exit 1
  rate token_transfer_underflow asm 1073741824 skip$x MYTHGPU_JIT_ASM_EXIT_SKIP=$x || exit 1
  rate suicide_kill asm 268435456 skip$x MYTHGPU_JIT_ASM_EXIT_SKIP=$x || exit 1
  rate walletlibrary_kill asm 268435456 skip$x MYTHGPU_JIT_ASM_EXIT_SKIP=$x || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_asm.py -m gpu -x -q -k "search or hit or needle or first" --timeout 200 --timeout-method thread > gpurun_out/r5s_pytest.log 2>&1 || true
tail -2 gpurun_out/r5s_pytest.log
cat gpurun_out/r5s_rates.jsonl
