# round 4, run Y: the new tests (many over virtual devices, tiled small n, UMUL widths, select CSE) then the asm/many suites
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_many.py -x -q --timeout 200 --timeout-method thread -k "not eval_workload" > gpurun_out/r4y_pytest.log 2>&1 || { tail -40 gpurun_out/r4y_pytest.log; exit 1; }
tail -2 gpurun_out/r4y_pytest.log
