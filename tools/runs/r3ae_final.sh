set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3ae_pytest.log 2>&1 || { tail -30 gpurun_out/r3ae_pytest.log; exit 1; }
tail -2 gpurun_out/r3ae_pytest.log
bash tools/profile.sh token_transfer_underflow jit 1073741824 || exit 1
cp gpurun_out/prof_token_transfer_underflow/pmc_token_transfer_underflow.json gpurun_out/pmc_headline_token_transfer_underflow.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc-dir gpurun_out > gpurun_out/r3ae_bench.json 2> gpurun_out/r3ae_bench.err || { tail -20 gpurun_out/r3ae_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3ae_bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['time_to_first_model_ms'], d['time_to_first_model_cold_ms'], d['time_to_first_model_hard']['cold_ms'])"
