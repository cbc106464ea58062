set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3x_pytest.log 2>&1 || { tail -30 gpurun_out/r3x_pytest.log; exit 1; }
tail -2 gpurun_out/r3x_pytest.log
bash tools/bench_all.sh || exit 1
cat gpurun_out/bench_all.jsonl | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['config']['workload'][:40], round(d['value']/1e9,1), d['roofline']['frac'], d['roofline']['valu_instructions_per_candidate'])"
