# round 4, run P4: the pushdown also for ITE results, and forced where the default is the compared
# value (MYTHGPU_EQ_PUSHDOWN=2) against the cost-checked default (=1): parity with =2, then A/B
set -o pipefail
mkdir -p gpurun_out
MYTHGPU_EQ_PUSHDOWN=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sweep or parity or gen3 or asm or jit or many" --deselect "tests/test_gpu_asm.py::test_asm_eval_workload_verdicts" --deselect "tests/test_gpu_jit.py::test_jit_vmtests_literals_as_runtime_inputs" > gpurun_out/r4p4_pytest.log 2>&1 || { tail -40 gpurun_out/r4p4_pytest.log; exit 1; }
tail -2 gpurun_out/r4p4_pytest.log
: > gpurun_out/r4p4.jsonl
for V in "p2=MYTHGPU_EQ_PUSHDOWN=2" "p1=MYTHGPU_EQ_PUSHDOWN=1" "p2b=MYTHGPU_EQ_PUSHDOWN=2" "p1b=MYTHGPU_EQ_PUSHDOWN=1"; do
  L=${V%%=*}; E=${V#*=}
  for EN in jit asm; do
    for W in walletlibrary_kill token_transfer_underflow; do
      env $E timeout -k 10 200 python bench.py --workload $W --engine $EN --candidates 268435456 --steps 10 --warmup 2 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4p4_b.json 2> gpurun_out/r4p4_b.err || { tail -5 gpurun_out/r4p4_b.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r4p4_b.json')); print(json.dumps({'variant': '$L', 'workload': '$W', 'engine': '$EN', 'value': d['value'], 'kernel_ms': d['roofline'].get('kernel_ms')}))" >> gpurun_out/r4p4.jsonl
    done
  done
done
cat gpurun_out/r4p4.jsonl
