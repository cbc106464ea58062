# round 5, run O (final): the whole GPU suite, smoke, the default bench line, the first tier's tiled
# C4 eval kernel's PMC under its final source
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --durations=8 --timeout 300 --timeout-method thread > gpurun_out/r5o_pytest.log 2>&1 || { tail -40 gpurun_out/r5o_pytest.log; exit 1; }
tail -2 gpurun_out/r5o_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5o_smoke.log 2>&1 || { tail -20 gpurun_out/r5o_smoke.log; exit 1; }
tail -1 gpurun_out/r5o_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r5o_bench.json 2> gpurun_out/r5o_bench.err || { tail -20 gpurun_out/r5o_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5o_bench.json").read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "roofline")}))
print(json.dumps({k: d["config"].get(k) for k in ("jit_tier", "jit_tier_rates", "jit_source_sha16")}))
for r in d.get("roofline_eval") or []:
    print(r["workload"][:12], r["kernel"][:34], r.get("soa_layout"), round(r["kernel_ms"], 4), round(r["hbm"]["frac"], 4), r.get("jit_source_sha16"))
h = d.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine")}))
print(json.dumps(d.get("cpu_baseline")))
PY
timeout -k 10 300 bash tools/profile_eval.sh walletlibrary_kill 4194304 1 1 || exit 1
head -c 700 gpurun_out/prof_evalasm_tiled_walletlibrary_kill/pmc_evalasm_tiled_walletlibrary_kill.json; echo
