set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3n_pytest.log 2>&1 || { tail -30 gpurun_out/r3n_pytest.log; exit 1; }
tail -2 gpurun_out/r3n_pytest.log
timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r3n_interp_latency.jsonl 2>&1 || exit 1
: > gpurun_out/r3n_interp_ab.jsonl
for W in suicide_kill token_transfer_underflow bectoken_batch_overflow walletlibrary_kill; do
  for H in 1 0; do
    MYTHGPU_INTERP_HOIST=$H timeout -k 10 120 python bench.py --workload $W --engine interp --candidates 4194304 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r3n_i.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3n_i.json')); print(json.dumps({'workload':'$W','hoist':$H,'value':d['value'],'kernel_ms':d['roofline']['kernel_ms'] if d.get('roofline') else None}))" >> gpurun_out/r3n_interp_ab.jsonl
  done
done
cat gpurun_out/r3n_interp_ab.jsonl
