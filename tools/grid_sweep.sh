#!/bin/bash
# GPU box: search-kernel time per launch-shape variant -> gpurun_out/grid_sweep.jsonl
#   VARIANTS="MYTHGPU_JIT_BPC=16 MYTHGPU_JIT_BPC=32,MYTHGPU_JIT_WAVES=4 ..." (comma-joined env settings)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/grid_sweep.jsonl
for W in ${WORKLOADS:-token_transfer_underflow walletlibrary_kill sha3_keyed_mapping bectoken_batch_overflow}; do
  N=268435456; [ "$W" = sha3_keyed_mapping ] && N=16777216
  for V in ${VARIANTS:-MYTHGPU_JIT_BPC=16 MYTHGPU_JIT_BPC=32 MYTHGPU_JIT_BPC=64}; do
    env ${V//,/ } timeout -k 10 120 python bench.py --workload $W --candidates $N --steps 5 --warmup 1 \
      --no-cpu-baseline --no-ttfm --no-stream > gpurun_out/gr.json 2> gpurun_out/gr_err.log || { tail -5 gpurun_out/gr_err.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/gr.json')); print(json.dumps({'workload': '$W', 'variant': '$V', 'kernel_ms': d['roofline']['kernel_ms'], 'value': d['value']}))" >> gpurun_out/grid_sweep.jsonl
  done
done
cat gpurun_out/grid_sweep.jsonl
