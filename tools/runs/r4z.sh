# round 4, run Z: interpreter 256-bit handlers load-all-then-store + generator constants in LDS; new tests;
# interpreter rates (LDS copy on / off) + one-wave latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "interp or sweep or parity or gen3 or capture or many or asm" --deselect "tests/test_gpu_asm.py::test_asm_eval_workload_verdicts" > gpurun_out/r4z_pytest.log 2>&1 || { tail -40 gpurun_out/r4z_pytest.log; exit 1; }
tail -2 gpurun_out/r4z_pytest.log
: > gpurun_out/r4z_interp.jsonl
for V in "ldsgen=" "noldsgen=MYTHGPU_INTERP_LDS_GEN=0"; do
  L=${V%%=*}; E=${V#*=}
  for W in token_transfer_underflow suicide_kill bectoken_batch_overflow walletlibrary_kill etherstore_reentrancy; do
    env $E timeout -k 10 200 python bench.py --workload $W --engine interp --candidates 4194304 --steps 20 --warmup 3 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4z_b.json 2> gpurun_out/r4z_b.err || { tail -5 gpurun_out/r4z_b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r4z_b.json')); print(json.dumps({'variant': '$L', 'workload': '$W', 'engine': 'interp', 'value': d['value'], 'kernel_ms': d['roofline'].get('kernel_ms')}))" >> gpurun_out/r4z_interp.jsonl
  done
done
cat gpurun_out/r4z_interp.jsonl
timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r4z_latency.jsonl 2>&1 || exit 1
tail -12 gpurun_out/r4z_latency.jsonl
