# round 4, run P3: the lookup-compare pushdown, also where the lookup stays (specialiser, compiled kernels' list): parity/sweep/asm
# tests, then search throughput O3 + first tier with and without it (MYTHGPU_EQ_PUSHDOWN=0), C1-C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sweep or parity or gen3 or asm or jit or many or replay or model" --deselect "tests/test_gpu_asm.py::test_asm_eval_workload_verdicts" > gpurun_out/r4p3_pytest.log 2>&1 || { tail -40 gpurun_out/r4p3_pytest.log; exit 1; }
tail -2 gpurun_out/r4p3_pytest.log
: > gpurun_out/r4p3.jsonl
for V in "push=MYTHGPU_EQ_PUSHDOWN=1" "nopush=MYTHGPU_EQ_PUSHDOWN=0"; do
  L=${V%%=*}; E=${V#*=}
  for EN in jit asm; do
    for W in token_transfer_underflow walletlibrary_kill suicide_kill etherstore_reentrancy; do
      env $E timeout -k 10 200 python bench.py --workload $W --engine $EN --steps 10 --warmup 2 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4p3_b.json 2> gpurun_out/r4p3_b.err || { tail -5 gpurun_out/r4p3_b.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r4p3_b.json')); print(json.dumps({'variant': '$L', 'workload': '$W', 'engine': '$EN', 'value': d['value'], 'kernel_ms': d['roofline'].get('kernel_ms')}))" >> gpurun_out/r4p3.jsonl
    done
  done
done
cat gpurun_out/r4p3.jsonl
