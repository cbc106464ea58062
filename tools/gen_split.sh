#!/bin/bash
# GPU box: generator vs evaluation VALU per candidate.  One rocprofv3 PMC pass per workload over the
# search kernel built with only the candidate generator (MYTHGPU_JIT_GEN_ONLY=1: its limbs XOR-folded
# into the verdict so nothing is dead); the full kernel's count is profiles/r03_pmc_<w>.json.
#   -> gpurun_out/gen_split.jsonl
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/gen_split.jsonl
for W in ${@:-suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill}; do
  D=gpurun_out/gsplit_$W; rm -rf $D; mkdir -p $D
  MYTHGPU_JIT_GEN_ONLY=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $D -o run --output-format csv -- \
    python3 bench.py --workload $W --candidates 268435456 --steps 2 --warmup 1 --no-cpu-baseline --no-ttfm --no-stream --no-eval > $D/log 2>&1 || { tail -5 $D/log; exit 1; }
  python3 - $D $W >> gpurun_out/gen_split.jsonl <<'PY'
import csv, glob, json, sys
from collections import defaultdict
d, w = sys.argv[1], sys.argv[2]
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mgj_search" in r.get("Kernel_Name", ""):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
top = max(x.get("SQ_INSTS_VALU", 0) for x in per.values())
full = [x for x in per.values() if x.get("SQ_INSTS_VALU", 0) >= 0.5 * top]
m = {k: sum(x[k] for x in full) / len(full) for k in full[0]}
n = 268435456
print(json.dumps({"workload": w, "gen_only_valu_per_candidate": m["SQ_INSTS_VALU"] * 64 / n,
                  "gen_only_salu_per_candidate": m["SQ_INSTS_SALU"] * 64 / n,
                  "gen_only_vmem_per_group": m["SQ_INSTS_VMEM_RD"] / (n / 64), "dispatches": len(full)}))
PY
done
cat gpurun_out/gen_split.jsonl
