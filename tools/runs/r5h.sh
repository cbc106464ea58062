# round 5, run H: rocprof kernel-trace stats + PMC passes of the headline kernel (C2 first tier,
# the tier bench.py chose in run G: source sha a6796c331431b736) at the headline size; then the eval
# kernels' rooflines with CONCAT/EXTRACT views in the first tier
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/profile.sh token_transfer_underflow asm 1073741824 || exit 1
cat gpurun_out/prof_token_transfer_underflow_asm/pmc_token_transfer_underflow.json | head -c 1500; echo
grep -A3 "mgj_search" gpurun_out/prof_token_transfer_underflow_asm/trace/*stats* | head -5
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --candidates 268435456 --no-cpu-baseline --no-stream --no-ttfm > gpurun_out/r5h_eval.json 2> gpurun_out/r5h_eval.err || { tail -20 gpurun_out/r5h_eval.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5h_eval.json").read().strip().splitlines()[-1])
for r in d.get("roofline_eval", []):
    print(r["workload"][:30], r["kernel"][:40], r.get("soa_layout"), round(r["kernel_ms"], 4), round(r["hbm"]["frac"], 4))
PY
