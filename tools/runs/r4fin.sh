# round 4, run FIN: the whole GPU suite at HEAD, smoke, bench (default line)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r4fin_pytest.log 2>&1 || { tail -40 gpurun_out/r4fin_pytest.log; exit 1; }
tail -20 gpurun_out/r4fin_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fin_smoke.log 2>&1 || { tail -20 gpurun_out/r4fin_smoke.log; exit 1; }
tail -3 gpurun_out/r4fin_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r4fin_bench.json 2> gpurun_out/r4fin_bench.err || { tail -20 gpurun_out/r4fin_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r4fin_bench.json')); print('value', d['value'], 'frac', d['roofline'].get('frac'), 'ttfm', d['time_to_first_model_ms'], d['time_to_first_model_cold_ms'], 'hard', d['time_to_first_model_hard']['cold_ms'], d['time_to_first_model_hard']['cold_engine'], 'cpu', d['cpu_baseline']['value'])"
