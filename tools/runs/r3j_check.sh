set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3j_pytest.log 2>&1 || { tail -30 gpurun_out/r3j_pytest.log; exit 1; }
tail -2 gpurun_out/r3j_pytest.log
timeout -k 10 300 python bench.py --pmc-dir gpurun_out --no-cpu-baseline > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err || { tail -20 gpurun_out/r3j_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3j_bench.json')); print(d['value'], d['time_to_first_model_ms'], json.dumps(d['time_to_first_model_hard']))"
bash tools/runs/r3_ab.sh r3j "base=" "nodskip=MYTHGPU_JIT_DELTA_SKIP=0" "novec=MYTHGPU_JIT_DICT_VEC=0" && cat gpurun_out/r3j_ab.jsonl
