#!/bin/bash
# GPU box: HEAD's GPU tests, the headline workload's PMC profile, the headline bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3i_pytest.log 2>&1 || { tail -30 gpurun_out/r3i_pytest.log; exit 1; }
tail -2 gpurun_out/r3i_pytest.log
bash tools/r3_prof.sh r3i token_transfer_underflow || exit 1
cp gpurun_out/pmc_token_transfer_underflow.json gpurun_out/r3i_pmc_token_transfer_underflow.json
timeout -k 10 400 python bench.py --pmc-dir gpurun_out > gpurun_out/r3i_bench.json 2> gpurun_out/r3i_bench.err || { tail -20 gpurun_out/r3i_bench.err; exit 1; }
cat gpurun_out/r3i_bench.json
