#!/bin/bash
# GPU box: each workload's search kernel with and without the constraint program
# (MYTHGPU_JIT_GEN_ONLY=1 keeps only the candidate generator) -> gpurun_out/gen_share.jsonl
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/gen_share.jsonl
for W in ${@:-suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill}; do
  for G in 0 1; do
    MYTHGPU_JIT_GEN_ONLY=$G timeout -k 10 120 python bench.py --workload $W --candidates 268435456 --steps 5 --warmup 1 \
      --no-cpu-baseline --no-ttfm --no-stream > gpurun_out/gs_${W}_${G}.json 2> gpurun_out/gs_err.log || { tail -5 gpurun_out/gs_err.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/gs_${W}_${G}.json')); print(json.dumps({'workload': '$W', 'gen_only': $G, 'kernel_ms': d['roofline']['kernel_ms'], 'value': d['value']}))" >> gpurun_out/gen_share.jsonl
  done
done
cat gpurun_out/gen_share.jsonl
