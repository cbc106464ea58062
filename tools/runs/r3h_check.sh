set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3h_pytest.log 2>&1 && tail -2 gpurun_out/r3h_pytest.log && \
bash tools/runs/r3_ab.sh r3ab6 "base=" "bpc16=MYTHGPU_JIT_BPC=16" && \
timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r3h_interp_latency.jsonl 2>&1 && \
MYTHGPU_INTERP_PREFETCH=0 timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r3h_interp_latency_nopf.jsonl 2>&1
