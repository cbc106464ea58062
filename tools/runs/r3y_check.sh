set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3y_pytest.log 2>&1 || { tail -30 gpurun_out/r3y_pytest.log; exit 1; }
tail -2 gpurun_out/r3y_pytest.log
timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r3y_interp_latency.jsonl 2>&1 || exit 1
grep workload gpurun_out/r3y_interp_latency.jsonl
timeout -k 10 200 python tools/latency_probe.py walletlibrary_kill > gpurun_out/r3y_latency_c4.json 2>&1 || exit 1
cat gpurun_out/r3y_latency_c4.json
