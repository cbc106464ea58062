# round 4, run O: eval kernels with watch rows (walking pointers) -- JIT eval + VMTests replay parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "eval or vmtests or capture or model" > gpurun_out/r4o_pytest.log 2>&1 || { tail -30 gpurun_out/r4o_pytest.log; exit 1; }
tail -2 gpurun_out/r4o_pytest.log
