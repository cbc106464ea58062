# round 5, run G: the whole GPU suite, smoke, the default bench line (the faster compiled tier for the
# headline, in-flight compile dedupe for the hard query), C5's hard query cold, then the PMC passes of
# the headline kernel the bench chose (tools/profile.sh at the headline size)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 300 --timeout-method thread > gpurun_out/r5g_pytest.log 2>&1 || { tail -40 gpurun_out/r5g_pytest.log; exit 1; }
tail -3 gpurun_out/r5g_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5g_smoke.log 2>&1 || { tail -20 gpurun_out/r5g_smoke.log; exit 1; }
tail -1 gpurun_out/r5g_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5g_bench.json 2> gpurun_out/r5g_bench.err || { tail -20 gpurun_out/r5g_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5g_bench.json").read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "roofline")}))
print(json.dumps({k: d["config"].get(k) for k in ("jit_tier", "jit_tier_rates", "jit_source_sha16")}))
h = d.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine")}), json.dumps(h.get("cold_timing")))
PY
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python bench.py --workload sha3_keyed_mapping --candidates 16777216 --steps 3 --no-stream --no-eval --no-cpu-baseline > gpurun_out/r5g_bench_c5.json 2> gpurun_out/r5g_bench_c5.err || { tail -20 gpurun_out/r5g_bench_c5.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5g_bench_c5.json").read().strip().splitlines()[-1])
print(json.dumps({k: d["config"].get(k) for k in ("jit_tier", "jit_tier_rates")}), d["value"])
h = d.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine")}), json.dumps(h.get("cold_timing")))
PY
grep -i "jit worker" gpurun_out/r5g_bench_c5.err | head -8
