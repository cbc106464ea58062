# round 4, run W2: BASELINE §4 rows at HEAD (every workload's PMC + bench line, 2^28; C5 2^24), then
# the first-tier column (asm engine, same sizes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/bench_all.sh || exit 1
: > gpurun_out/bench_all_asm.jsonl
for W in suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill; do
  timeout -k 10 200 python bench.py --workload $W --engine asm --candidates 268435456 --steps 10 --warmup 2 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/ba_$W.json 2> gpurun_out/ba_$W.err || { tail -5 gpurun_out/ba_$W.err; exit 1; }
  cat gpurun_out/ba_$W.json >> gpurun_out/bench_all_asm.jsonl
done
python3 -c "
import json
for f in ('gpurun_out/bench_all.jsonl', 'gpurun_out/bench_all_asm.jsonl'):
    for l in open(f):
        d = json.loads(l); r = d['roofline']
        print(f[-10:], d['config']['workload'][:40], round(d['value']/1e9, 1), r.get('valu_instructions_per_candidate'), r.get('frac'), d.get('cpu_baseline', {}).get('value') if d.get('cpu_baseline') else None)
"
