set -o pipefail
mkdir -p gpurun_out
bash tools/profile.sh token_transfer_underflow jit 1073741824 || exit 1
cp gpurun_out/prof_token_transfer_underflow/pmc_token_transfer_underflow.json gpurun_out/pmc_headline_token_transfer_underflow.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc-dir gpurun_out > gpurun_out/r3ab_bench.json 2> gpurun_out/r3ab_bench.err || { tail -20 gpurun_out/r3ab_bench.err; exit 1; }
cat gpurun_out/r3ab_bench.json
