set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "jit or sweep or gen3" > gpurun_out/r3t_pytest.log 2>&1 || { tail -30 gpurun_out/r3t_pytest.log; exit 1; }
tail -2 gpurun_out/r3t_pytest.log
: > gpurun_out/r3t_ab.jsonl
for V in "pf=" "nopf=MYTHGPU_JIT_PREFETCH=0"; do
  L=${V%%=*}; E=${V#*=}
  for W in bectoken_batch_overflow etherstore_reentrancy token_transfer_underflow; do
    env $E timeout -k 10 300 python bench.py --workload $W --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r3t_b.json 2> gpurun_out/r3t_b.err || { tail -5 gpurun_out/r3t_b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/r3t_b.json')); print(json.dumps({'variant': '$L', 'workload': '$W', 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'sha': d['config']['jit_source_sha16']}))" >> gpurun_out/r3t_ab.jsonl
  done
done
cat gpurun_out/r3t_ab.jsonl
