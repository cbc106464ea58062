# round 5, run A: baseline at the round's start — whole GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5a_pytest.log 2>&1 || { tail -40 gpurun_out/r5a_pytest.log; exit 1; }
tail -3 gpurun_out/r5a_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5a_smoke.log 2>&1 || { tail -20 gpurun_out/r5a_smoke.log; exit 1; }
tail -3 gpurun_out/r5a_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || { tail -20 gpurun_out/r5a_bench.err; exit 1; }
tail -c 600 gpurun_out/r5a_bench.json
