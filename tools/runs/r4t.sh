# round 4, run T: every workload's O3 kernel (PMC + bench at 2^28, C5 2^24) and first-tier rate, for BASELINE.md section 4
set -o pipefail
mkdir -p gpurun_out
bash tools/bench_all.sh || exit 1
: > gpurun_out/r4t_asm.jsonl
for W in suicide_kill token_transfer_underflow etherstore_reentrancy walletlibrary_kill; do
  timeout -k 10 200 python bench.py --workload $W --engine asm --candidates 268435456 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4t_a.json 2> gpurun_out/r4t_a.err || { tail -5 gpurun_out/r4t_a.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4t_a.json')); print(json.dumps({'workload': '$W', 'engine': 'asm', 'value': d['value'], 'kernel_ms': d['roofline'].get('kernel_ms')}))" >> gpurun_out/r4t_asm.jsonl
done
cat gpurun_out/r4t_asm.jsonl
python3 -c "
import json
for l in open('gpurun_out/bench_all.jsonl'):
    d=json.loads(l); print(d['config']['workload'][:40], d['value'], d['roofline'].get('frac'), d['roofline'].get('valu_instructions_per_candidate'))"
