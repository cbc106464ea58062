# round 4, run C: first-tier parity after the literal pool; its rate; the bench line (hard needle cold)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_asm.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1 || { tail -30 gpurun_out/r4c_pytest.log; exit 1; }
tail -2 gpurun_out/r4c_pytest.log
timeout -k 10 120 python tools/launch_size.py token_transfer_underflow --asm > gpurun_out/r4c_launch_size_asm.jsonl || exit 1
cat gpurun_out/r4c_launch_size_asm.jsonl
timeout -k 10 400 python bench.py --gpus 1 --no-cpu-baseline > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err || { tail -20 gpurun_out/r4c_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r4c_bench.json"))
print("value", d["value"], "ttfm", d["time_to_first_model_ms"], d["time_to_first_model_cold_ms"])
print("hard", json.dumps(d["time_to_first_model_hard"])[:1500])
print("asm", d["jit_asm_tier"])
print("stream", {k: d["dropin_stream"][k] for k in ("queries", "stream_s", "engines")} if d["dropin_stream"] else None)
PY
