set -o pipefail
mkdir -p gpurun_out
bash tools/bench_all.sh || exit 1
cat gpurun_out/bench_all.jsonl | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['config']['workload'][:40], round(d['value']/1e9,1), d['roofline']['frac'], d['roofline']['valu_instructions_per_candidate'])"
