# round 5, run B: the first tier with the whole vocabulary on the GPU — the asm parity suite (200 random
# programs for gen verdicts and for eval watch rows, every workload incl. C5), then C5 through the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_jit.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5b_pytest.log 2>&1 || { tail -40 gpurun_out/r5b_pytest.log; exit 1; }
tail -3 gpurun_out/r5b_pytest.log
timeout -k 10 300 python bench.py --workload sha3_keyed_mapping --candidates 16777216 --steps 5 --no-stream --no-eval --no-cpu-baseline > gpurun_out/r5b_bench_c5.json 2> gpurun_out/r5b_bench_c5.err || { tail -20 gpurun_out/r5b_bench_c5.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5b_bench_c5.json").read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step")}))
print(json.dumps(d.get("jit_asm_tier")))
h = d.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine", "index", "candidates")}), json.dumps(h.get("cold_timing")))
PY
