# round 4, run L: tiled SoA eval kernels (O3 + first tier)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_many.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4l_pytest.log 2>&1 || { tail -30 gpurun_out/r4l_pytest.log; exit 1; }
tail -2 gpurun_out/r4l_pytest.log
timeout -k 10 400 python bench.py --gpus 1 --no-cpu-baseline > gpurun_out/r4l_bench.json 2> gpurun_out/r4l_bench.err || { tail -20 gpurun_out/r4l_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r4l_bench.json"))
print("value", d["value"], "ttfm", d["time_to_first_model_ms"], d["time_to_first_model_cold_ms"])
h = d["time_to_first_model_hard"]
print("hard", h["cold_ms"], h["cold_engine"], h["warm_ms"], h["cold_timing"])
print("asm", d["jit_asm_tier"])
for e in d["roofline_eval"]:
    print(e.get("kernel"), e.get("workload")[:20], e.get("kernel_ms"), (e.get("hbm") or {}).get("frac"), e.get("soa_rows_read"), e.get("unsupported", "")[:80])
PY
echo done
echo done
