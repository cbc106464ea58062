# watch-free eval kernels walk the SoA rows with one pointer: GPU suite, then the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 240 --timeout-method thread > gpurun_out/r3za_pytest.log 2>&1 || { tail -30 gpurun_out/r3za_pytest.log; exit 1; }
tail -3 gpurun_out/r3za_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r3za_bench.json 2> gpurun_out/r3za_bench.err || { tail -20 gpurun_out/r3za_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3za_bench.json')); print(d['value'], d['roofline']['frac'], [(e['workload'][:3], e['soa_rows_read'], e['kernel_ms'], e['hbm']['frac']) for e in d['roofline_eval']])"
