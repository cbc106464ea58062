# round 5, run P (final): the whole GPU suite, smoke, the default bench line, the first tier's tiled
# C4 eval PMC under its final source, then blocks per CU for the first tier's C3 search kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --durations=8 --timeout 300 --timeout-method thread > gpurun_out/r5p_pytest.log 2>&1 || { tail -40 gpurun_out/r5p_pytest.log; exit 1; }
tail -2 gpurun_out/r5p_pytest.log
grep -E "vmtests" gpurun_out/r5p_pytest.log | head -3
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5p_smoke.log 2>&1 || { tail -20 gpurun_out/r5p_smoke.log; exit 1; }
tail -1 gpurun_out/r5p_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r5p_bench.json 2> gpurun_out/r5p_bench.err || { tail -20 gpurun_out/r5p_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5p_bench.json").read().strip().splitlines()[-1])
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
: > gpurun_out/r5p_rates.jsonl
rate() {  # workload engine candidates tag [env...]
  local w=$1 e=$2 n=$3 tag=$4; shift 4
  env "$@" timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5p_b.json 2> gpurun_out/r5p_b.err || { tail -20 gpurun_out/r5p_b.err; return 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/r5p_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'tag': '$tag', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5p_rates.jsonl
}
rate bectoken_batch_overflow jit 268435456 o3 || exit 1
for b in 32 64 128; do rate bectoken_batch_overflow asm 268435456 bpc$b MYTHGPU_JIT_BPC=$b || exit 1; done
rate bectoken_batch_overflow asm 268435456 no_mulshare MYTHGPU_JIT_ASM_NO_MULSHARE=1 || exit 1
cat gpurun_out/r5p_rates.jsonl
