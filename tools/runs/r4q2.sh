set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_many.py tests/test_gpu_asm.py -x -q --timeout 200 --timeout-method thread -k "eval or many or tiled or umul" --deselect "tests/test_gpu_asm.py::test_asm_eval_workload_verdicts" > gpurun_out/r4q2_pytest.log 2>&1 || { tail -30 gpurun_out/r4q2_pytest.log; exit 1; }
tail -2 gpurun_out/r4q2_pytest.log
