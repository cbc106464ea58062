#!/bin/bash
# GPU-box check: build already done in-tree (the .so travels with the snapshot).
#   tools/gpu_check.sh [tag] [pytest -k expr]   -> gpurun_out/<tag>_{pytest,bench}.log
set -o pipefail
T=${1:-chk}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 240 --timeout-method thread -k "$K" > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
fi
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
