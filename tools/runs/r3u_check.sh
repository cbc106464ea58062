set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "jit or sweep or gen3 or capture or solver" > gpurun_out/r3u_pytest.log 2>&1 || { tail -30 gpurun_out/r3u_pytest.log; exit 1; }
tail -2 gpurun_out/r3u_pytest.log
bash tools/runs/r3_ab.sh r3u "nobarrier=" && cat gpurun_out/r3u_ab.jsonl
