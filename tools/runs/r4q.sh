# round 4, run Q: eval launch shape (blocks per CU / groups per wave) for the eval kernels
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r4q_eval_grid.jsonl
for V in "d=" "mg0=MYTHGPU_JIT_MIN_GROUPS=0" "mg4=MYTHGPU_JIT_MIN_GROUPS=4" "bpc2=MYTHGPU_JIT_BPC=2" "bpc8=MYTHGPU_JIT_BPC=8"; do
  L=${V%%=*}; E=${V#*=}
  for C in "walletlibrary_kill 1 1" "walletlibrary_kill 0 1" "walletlibrary_kill 0 0" "token_transfer_underflow 0 1" "token_transfer_underflow 1 1"; do
    set -- $C
    env $E timeout -k 10 120 python tools/eval_probe.py $1 4194304 5 $2 $3 > gpurun_out/r4q_p.json 2> gpurun_out/r4q_p.err || { tail -5 gpurun_out/r4q_p.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4q_p.json').read().splitlines()[-1])['eval']; print(json.dumps({'variant': '$L', 'workload': '$1', 'asm': $2, 'tiled': $3, 'kernel_ms': round(d['kernel_ms'],4), 'hbm_frac': round(d['hbm']['frac'],4)}))" >> gpurun_out/r4q_eval_grid.jsonl
  done
done
cat gpurun_out/r4q_eval_grid.jsonl
