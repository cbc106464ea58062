# round 5, run N: the GPU suite's JIT and first-tier files (spills to LDS, -O0 read-back fallbacks,
# UMUL_NOOVF/MUL product sharing, row page bases cached), blocks per CU for the first tier's search
# kernels against O3 (C3, C1, C4 at 2^28), the eval kernels' queue modes, the VMTests replay per phase
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_asm.py -m gpu -x -q --durations=6 --timeout 300 --timeout-method thread > gpurun_out/r5n_pytest.log 2>&1 || { tail -40 gpurun_out/r5n_pytest.log; exit 1; }
tail -9 gpurun_out/r5n_pytest.log
: > gpurun_out/r5n_rates.jsonl
rate() {  # workload engine candidates tag [env...]
  local w=$1 e=$2 n=$3 tag=$4; shift 4
  env "$@" timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5n_b.json 2> gpurun_out/r5n_b.err || { tail -20 gpurun_out/r5n_b.err; return 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/r5n_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'tag': '$tag', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5n_rates.jsonl
}
rate bectoken_batch_overflow jit 268435456 o3 || exit 1
for b in 16 32 64 128; do rate bectoken_batch_overflow asm 268435456 bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
rate bectoken_batch_overflow asm 268435456 no_mulshare MYTHGPU_JIT_ASM_NO_MULSHARE=1 || exit 1
for w in suicide_kill walletlibrary_kill; do
  rate $w jit 268435456 o3 || exit 1
  for b in 32 64 128; do rate $w asm 268435456 bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
done
cat gpurun_out/r5n_rates.jsonl
timeout -k 10 600 python tools/eval_glds_sweep.py > gpurun_out/r5n_eval.jsonl 2> gpurun_out/r5n_eval.err || { tail -20 gpurun_out/r5n_eval.err; exit 1; }
cat gpurun_out/r5n_eval.jsonl
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python tools/vmtests_timing.py 400 > gpurun_out/r5n_vmt.json 2> gpurun_out/r5n_vmt.err || { tail -5 gpurun_out/r5n_vmt.err; exit 0; }
cat gpurun_out/r5n_vmt.json
