set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3w_pytest.log 2>&1 || { tail -30 gpurun_out/r3w_pytest.log; exit 1; }
tail -2 gpurun_out/r3w_pytest.log
bash tools/runs/r3_ab.sh r3w "bpc32=" "bpc64=MYTHGPU_JIT_BPC=64" && cat gpurun_out/r3w_ab.jsonl
: > gpurun_out/r3w_interp.jsonl
for W in suicide_kill token_transfer_underflow bectoken_batch_overflow; do
  timeout -k 10 120 python bench.py --workload $W --engine interp --candidates 4194304 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r3w_i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3w_i.json')); print(json.dumps({'engine':'interp','workload':'$W','value':d['value']}))" >> gpurun_out/r3w_interp.jsonl
done
cat gpurun_out/r3w_interp.jsonl
