# round 5, run T (final): the end-of-wave hit-word read on by default — the whole GPU suite, smoke,
# the default bench line, and the headline kernel's rocprof + PMC passes under its new source
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --durations=4 --timeout 300 --timeout-method thread > gpurun_out/r5t_pytest.log 2>&1 || { tail -40 gpurun_out/r5t_pytest.log; exit 1; }
tail -2 gpurun_out/r5t_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5t_smoke.log 2>&1 || { tail -20 gpurun_out/r5t_smoke.log; exit 1; }
tail -1 gpurun_out/r5t_smoke.log
timeout -k 10 420 bash tools/profile.sh token_transfer_underflow asm 1073741824 || exit 1
head -c 400 gpurun_out/prof_token_transfer_underflow_asm/pmc_token_transfer_underflow.json; echo
timeout -k 10 400 python bench.py > gpurun_out/r5t_bench.json 2> gpurun_out/r5t_bench.err || { tail -20 gpurun_out/r5t_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5t_bench.json").read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "roofline")}))
print(json.dumps({k: d["config"].get(k) for k in ("jit_tier", "jit_tier_rates", "jit_source_sha16")}))
PY
