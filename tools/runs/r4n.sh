# round 4, run N: interpreter k-groups (KG groups per wave per program pass): parity + throughput per KG
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "interp or sweep or parity or gen3 or capture or early or many or multidevice" > gpurun_out/r4n_pytest.log 2>&1 || { tail -30 gpurun_out/r4n_pytest.log; exit 1; }
tail -2 gpurun_out/r4n_pytest.log
: > gpurun_out/r4n_kg.jsonl
for KG in 1 2 4; do
  for W in token_transfer_underflow suicide_kill bectoken_batch_overflow walletlibrary_kill; do
    MYTHGPU_INTERP_KG=$KG timeout -k 10 200 python bench.py --workload $W --engine interp --candidates 4194304 --steps 20 --warmup 3 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4n_b.json 2> gpurun_out/r4n_b.err || { tail -5 gpurun_out/r4n_b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r4n_b.json')); print(json.dumps({'kg': $KG, 'workload': '$W', 'value': d['value'], 'kernel_ms': d['roofline'].get('kernel_ms')}))" >> gpurun_out/r4n_kg.jsonl
  done
done
cat gpurun_out/r4n_kg.jsonl
MYTHGPU_INTERP_KG=2 timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r4n_latency_kg2.jsonl 2>&1 || exit 1
tail -6 gpurun_out/r4n_latency_kg2.jsonl
