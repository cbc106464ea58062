# round 4, run B2: the first tier's Bool lookups on lane masks (MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP=1: limbs):
# asm tests (eval verdicts included), A/B of the asm search kernel, the asm eval PMC at the new
# sources (into profiles/ on the box), the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_sweep.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4b2_pytest.log 2>&1 || { tail -40 gpurun_out/r4b2_pytest.log; exit 1; }
tail -2 gpurun_out/r4b2_pytest.log
: > gpurun_out/r4b2.jsonl
for V in "mask=MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP=0" "limb=MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP=1" "maskb=MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP=0" "limbb=MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP=1"; do
  L=${V%%=*}; E=${V#*=}
  for W in walletlibrary_kill token_transfer_underflow; do
    env $E timeout -k 10 200 python bench.py --workload $W --engine asm --candidates 268435456 --steps 10 --warmup 2 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4b2_b.json 2> gpurun_out/r4b2_b.err || { tail -5 gpurun_out/r4b2_b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r4b2_b.json')); print(json.dumps({'variant': '$L', 'workload': '$W', 'engine': 'asm', 'value': d['value'], 'kernel_ms': d['roofline'].get('kernel_ms')}))" >> gpurun_out/r4b2.jsonl
  done
done
cat gpurun_out/r4b2.jsonl
for W in token_transfer_underflow walletlibrary_kill; do
  bash tools/profile_eval.sh $W 4194304 1 1 || { echo "profile evalasm tiled $W failed"; exit 1; }
  cp gpurun_out/prof_evalasm_tiled_$W/pmc_evalasm_tiled_$W.json profiles/r04b2_pmc_evalasm_tiled_$W.json
done
mkdir -p gpurun_out/b2 && cp profiles/r04b2_* gpurun_out/b2/
timeout -k 10 500 python bench.py > gpurun_out/r4b2_bench.json 2> gpurun_out/r4b2_bench.err || { tail -20 gpurun_out/r4b2_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r4b2_bench.json')); print('value', d['value'], 'frac', d['roofline'].get('frac'), 'traffic', d['roofline'].get('traffic'), 'hard', d['time_to_first_model_hard']['cold_ms'], d['time_to_first_model_hard']['cold_engine'])
for e in d['roofline_eval']: print(e['kernel'], e['soa_layout'], round(e['hbm']['frac'], 3), e['hbm'].get('traffic'))"
