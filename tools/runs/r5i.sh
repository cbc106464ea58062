# round 5, run I: the whole GPU suite with LDS-staged eval rows (global_load_lds_dword) and the greedy
# constraint order, then the tiled first-tier eval kernel's HBM rate against its row queue
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 300 --timeout-method thread > gpurun_out/r5i_pytest.log 2>&1 || { tail -40 gpurun_out/r5i_pytest.log; exit 1; }
tail -3 gpurun_out/r5i_pytest.log
timeout -k 10 600 python tools/eval_glds_sweep.py > gpurun_out/r5i_eval_glds.jsonl 2> gpurun_out/r5i_eval_glds.err || { tail -20 gpurun_out/r5i_eval_glds.err; exit 1; }
cat gpurun_out/r5i_eval_glds.jsonl
