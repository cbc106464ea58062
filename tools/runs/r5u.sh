# round 5, run U: C5's hard query cold and warm at the final sources
set -o pipefail
mkdir -p gpurun_out
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python bench.py --workload sha3_keyed_mapping --candidates 16777216 --steps 3 --no-stream --no-eval --no-cpu-baseline > gpurun_out/r5u_bench_c5.json 2> gpurun_out/r5u_bench_c5.err || { tail -20 gpurun_out/r5u_bench_c5.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5u_bench_c5.json").read().strip().splitlines()[-1])
print(json.dumps({k: d["config"].get(k) for k in ("jit_tier", "jit_tier_rates")}), d["value"])
h = d.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine")}), json.dumps(h.get("cold_timing")))
PY
