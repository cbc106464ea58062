#!/bin/bash
# Throughput of one workload's JIT kernel under compiler / launch variants (GPU box).
#   tools/jit_sweep.sh <workload> [label=ENV=value ...] -> gpurun_out/sweep_<workload>.jsonl
W=${1:-token_transfer_underflow}; shift
O=gpurun_out/sweep_$W.jsonl
mkdir -p gpurun_out; : > $O
run() {  # label, env...
  local label=$1; shift
  env "$@" AMD_COMGR_CACHE=0 timeout -k 10 120 python bench.py --workload $W --no-cpu-baseline --no-ttfm --no-stream --no-eval --steps 20 > /tmp/sw.json 2>/tmp/sw.err || { echo "{\"label\": \"$label\", \"error\": true}" >> $O; return 0; }
  python3 -c "import json,sys; d=json.load(open('/tmp/sw.json')); print(json.dumps({'label': sys.argv[1], 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'compile_ms': d['config']['jit_compile_ms_cold']}))" "$label" >> $O
}
if [ $# -eq 0 ]; then
  run base
  run bpc16 MYTHGPU_JIT_BPC=16
  run maxilp "MYTHGPU_JIT_EXTRA=-mllvm --amdgpu-sched-strategy=max-ilp"
  run O2 MYTHGPU_JIT_OPT=2
else
  run base
  for v in "$@"; do run "${v%%=*}" "${v#*=}"; done
fi
cat $O
