#!/bin/bash
# GPU box: A/B of the JIT search kernel under compiler-option / emission variants (env), every
# C1-C4 workload, no PMC.   tools/r3_ab.sh <tag> "<label>=<env assignments>" ...
set -o pipefail
T=${1:-r3ab}; shift
mkdir -p gpurun_out
: > gpurun_out/${T}_ab.jsonl
for V in "$@"; do
  L=${V%%=*}; E=${V#*=}
  for W in suicide_kill token_transfer_underflow bectoken_batch_overflow walletlibrary_kill; do
    env $E timeout -k 10 300 python bench.py --workload $W --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/${T}_${L}_$W.json 2> gpurun_out/${T}_${L}_$W.err || { tail -5 gpurun_out/${T}_${L}_$W.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_${L}_$W.json')); print(json.dumps({'variant': '$L', 'env': '$E', 'workload': '$W', 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'sha': d['config']['jit_source_sha16']}))" >> gpurun_out/${T}_ab.jsonl
  done
done
