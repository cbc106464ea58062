set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3s_pytest.log 2>&1 || { tail -30 gpurun_out/r3s_pytest.log; exit 1; }
tail -2 gpurun_out/r3s_pytest.log
bash tools/profile.sh token_transfer_underflow interp 4194304 || exit 1
timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r3s_interp_latency.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/latency_probe.py > gpurun_out/r3s_latency.jsonl 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.err || { tail -20 gpurun_out/r3s_bench.err; exit 1; }
cat gpurun_out/r3s_bench.json
