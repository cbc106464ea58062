# round 4, run J: eval kernels' HBM rate against the SoA shape (row stride, queue depth)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/eval_sweep.py > gpurun_out/r4j_eval_sweep.jsonl 2> gpurun_out/r4j_eval_sweep.err || { tail -20 gpurun_out/r4j_eval_sweep.err; exit 1; }
cat gpurun_out/r4j_eval_sweep.jsonl
