set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3aa_bench.json 2> gpurun_out/r3aa_bench.err || { tail -20 gpurun_out/r3aa_bench.err; exit 1; }
cat gpurun_out/r3aa_bench.json
