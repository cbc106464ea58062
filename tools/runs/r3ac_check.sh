set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3ac_pytest.log 2>&1 || { tail -30 gpurun_out/r3ac_pytest.log; exit 1; }
tail -2 gpurun_out/r3ac_pytest.log
timeout -k 10 400 python bench.py > gpurun_out/r3ac_bench.json 2> gpurun_out/r3ac_bench.err || { tail -20 gpurun_out/r3ac_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3ac_bench.json')); print(d['value'], d['roofline']['frac'], d['config']['jit_compile_ms_cold'], d['time_to_first_model_ms'], d['time_to_first_model_cold_ms'], d['time_to_first_model_hard']['cold_ms'], json.dumps(d['dropin_stream']))"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ac_smoke.log 2>&1 || { tail -20 gpurun_out/r3ac_smoke.log; exit 1; }
tail -1 gpurun_out/r3ac_smoke.log
