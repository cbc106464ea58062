#!/bin/bash
# The round's full GPU check, as the driver runs it plus the evidence the bench line cites:
# the whole `-m gpu` suite, smoke(), the headline kernel's rocprof kernel trace + PMC passes, the
# default bench line, and C5's hard query.  Usage (on the GPU box): tools/full_run.sh <tag>
#   -> gpurun_out/<tag>_{pytest.log,smoke.log,bench.json,bench_c5.json} and
#      gpurun_out/prof_token_transfer_underflow_asm/ (copy the summaries judged into profiles/; the
#      headline PMC summary is also placed in the box's profiles/ before the bench reads it)
set -o pipefail
T=${1:-run}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=6 --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 420 bash tools/profile.sh token_transfer_underflow asm 1073741824 || exit 1
# the bench line's roofline reads the PMC summary of its kernel from profiles/ (matched by source SHA)
cp gpurun_out/prof_token_transfer_underflow_asm/pmc_token_transfer_underflow.json profiles/${T}_pmc_asm_token_transfer_underflow.json || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python bench.py --workload sha3_keyed_mapping --candidates 16777216 --steps 3 --no-stream --no-eval --no-cpu-baseline > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err || { tail -20 gpurun_out/${T}_bench_c5.err; exit 1; }
python - "$T" <<'PY'
import json, sys
t = sys.argv[1]
d = json.loads(open(f"gpurun_out/{t}_bench.json").read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "roofline")}))
print(json.dumps({k: d["config"].get(k) for k in ("jit_tier", "jit_tier_rates", "jit_source_sha16")}))
c = json.loads(open(f"gpurun_out/{t}_bench_c5.json").read().strip().splitlines()[-1])
h = c.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine")}), json.dumps(h.get("cold_timing")))
PY
