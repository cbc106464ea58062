# round 4, run D: every GPU test, JIT compile phases (both tiers), the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4d_pytest.log 2>&1 || { tail -30 gpurun_out/r4d_pytest.log; exit 1; }
tail -2 gpurun_out/r4d_pytest.log
timeout -k 10 300 python tools/jit_phases.py > gpurun_out/r4d_jit_phases.jsonl 2> gpurun_out/r4d_jit_phases.err || { tail -20 gpurun_out/r4d_jit_phases.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_bench.err || { tail -20 gpurun_out/r4d_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r4d_bench.json"))
print("value", d["value"], "frac", d["roofline"]["frac"], "ttfm", d["time_to_first_model_ms"], d["time_to_first_model_cold_ms"])
h = d["time_to_first_model_hard"]
print("hard", h["cold_ms"], h["cold_engine"], h["warm_ms"], h["warm_engine"], h["cold_timing"])
print("asm", d["jit_asm_tier"])
print("cpu", d["cpu_baseline"])
PY
bash tools/profile.sh token_transfer_underflow asm 268435456 || exit 1
cp gpurun_out/prof_token_transfer_underflow_asm/pmc_token_transfer_underflow.json gpurun_out/pmc_asm_token_transfer_underflow.json
python3 -c "import json; d=json.load(open('gpurun_out/pmc_asm_token_transfer_underflow.json')); print(json.dumps(d.get('derived')))"
