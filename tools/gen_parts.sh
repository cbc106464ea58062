#!/bin/bash
# GPU box: search-kernel time of the generator alone, split by generator kind
# (MYTHGPU_JIT_GEN_ONLY=1 + MYTHGPU_JIT_GEN_KIND=k) -> gpurun_out/gen_parts.jsonl
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/gen_parts.jsonl
W=${1:-token_transfer_underflow}
for K in all 1 2 3 4 5; do
  if [ "$K" = all ]; then E="MYTHGPU_JIT_GEN_ONLY=1"; else E="MYTHGPU_JIT_GEN_ONLY=1 MYTHGPU_JIT_GEN_KIND=$K"; fi
  env $E timeout -k 10 120 python bench.py --workload $W --candidates 268435456 --steps 5 --warmup 1 \
    --no-cpu-baseline --no-ttfm --no-stream > gpurun_out/gp.json 2> gpurun_out/gp_err.log || { tail -5 gpurun_out/gp_err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/gp.json')); print(json.dumps({'workload': '$W', 'gen_kind': '$K', 'kernel_ms': d['roofline']['kernel_ms']}))" >> gpurun_out/gen_parts.jsonl
done
cat gpurun_out/gen_parts.jsonl
