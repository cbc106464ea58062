# round 4, run A: HEAD after the ADVICE fixes — GPU tests, the bench line, the JIT's compile phases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1 || { tail -30 gpurun_out/r4a_pytest.log; exit 1; }
tail -2 gpurun_out/r4a_pytest.log
timeout -k 10 300 python tools/jit_phases.py > gpurun_out/r4a_jit_phases.jsonl 2> gpurun_out/r4a_jit_phases.err || { tail -20 gpurun_out/r4a_jit_phases.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || { tail -20 gpurun_out/r4a_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4a_bench.json')); print(d['value'], d['roofline']['frac'], d['time_to_first_model_ms'], d['time_to_first_model_cold_ms'], d['time_to_first_model_hard']['cold_ms'])"
