set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3z_pytest.log 2>&1 || { tail -30 gpurun_out/r3z_pytest.log; exit 1; }
tail -2 gpurun_out/r3z_pytest.log
: > gpurun_out/r3z_interp_ab.jsonl
for T in 1 0; do
  for W in bectoken_batch_overflow sha3_keyed_mapping token_transfer_underflow; do
    MYTHGPU_INTERP_TIERS=$T timeout -k 10 120 python bench.py --workload $W --engine interp --candidates 4194304 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r3z_i.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3z_i.json')); print(json.dumps({'engine':'interp','workload':'$W','tiers':$T,'value':d['value']}))" >> gpurun_out/r3z_interp_ab.jsonl
  done
  MYTHGPU_INTERP_TIERS=$T timeout -k 10 300 python bench.py --no-stream --no-eval --no-cpu-baseline > gpurun_out/r3z_b$T.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3z_b$T.json')); print(json.dumps({'tiers':$T,'hard':d['time_to_first_model_hard']}))" >> gpurun_out/r3z_interp_ab.jsonl
done
cat gpurun_out/r3z_interp_ab.jsonl
