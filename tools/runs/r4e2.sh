# round 4, run E2: first tier with the equality-difference cache (default) against without it
# (MYTHGPU_JIT_ASM_NO_EQ_CACHE=1): asm tests, then C2/C4 search throughput and VALU per candidate
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_many.py -x -q --timeout 200 --timeout-method thread -k "not eval_workload" > gpurun_out/r4e2_pytest.log 2>&1 || { tail -40 gpurun_out/r4e2_pytest.log; exit 1; }
tail -2 gpurun_out/r4e2_pytest.log
: > gpurun_out/r4e2.jsonl
for V in "eqcache=MYTHGPU_JIT_ASM_NO_EQ_CACHE=0" "noeqcache=MYTHGPU_JIT_ASM_NO_EQ_CACHE=1"; do
  L=${V%%=*}; E=${V#*=}
  for W in token_transfer_underflow walletlibrary_kill suicide_kill etherstore_reentrancy; do
    env $E timeout -k 10 200 python bench.py --workload $W --engine asm --steps 10 --warmup 2 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4e2_b.json 2> gpurun_out/r4e2_b.err || { tail -5 gpurun_out/r4e2_b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r4e2_b.json')); print(json.dumps({'variant': '$L', 'workload': '$W', 'engine': 'asm', 'value': d['value'], 'kernel_ms': d['roofline'].get('kernel_ms')}))" >> gpurun_out/r4e2.jsonl
  done
  for W in token_transfer_underflow walletlibrary_kill; do
    env $E bash tools/profile.sh $W asm 268435456 > /dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/prof_${W}_asm/pmc_$W.json')); print(json.dumps({'variant': '$L', 'workload': '$W', 'valu_per_cand': d['derived']['valu_wave_instructions_per_candidate'], 'salu_per_cand': d['derived']['salu_instructions_per_candidate']}))" >> gpurun_out/r4e2.jsonl
  done
done
cat gpurun_out/r4e2.jsonl
