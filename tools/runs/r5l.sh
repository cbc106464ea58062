# round 5, run L: the VMTests read-back replay with LDS spills and -O0 fallbacks (per phase, all
# vectors), then the GPU suite's JIT and first-tier files
set -o pipefail
mkdir -p gpurun_out
MYTHGPU_JIT_TIMING=1 timeout -k 10 400 python tools/vmtests_timing.py 400 > gpurun_out/r5l_vmt.json 2> gpurun_out/r5l_vmt.err || { tail -5 gpurun_out/r5l_vmt.err; exit 1; }
cat gpurun_out/r5l_vmt.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_asm.py -m gpu -x -q --durations=6 --timeout 300 --timeout-method thread > gpurun_out/r5l_pytest.log 2>&1 || { tail -40 gpurun_out/r5l_pytest.log; exit 1; }
tail -9 gpurun_out/r5l_pytest.log
