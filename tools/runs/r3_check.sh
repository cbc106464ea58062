#!/bin/bash
# GPU box: the -m gpu suite, then every workload's JIT kernel rate (no PMC), then the headline
# bench line.  -> gpurun_out/<tag>_{pytest.log,workloads.jsonl,bench.json}
set -o pipefail
T=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
: > gpurun_out/${T}_workloads.jsonl
for W in suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill sha3_keyed_mapping; do
  N=268435456; [ "$W" = sha3_keyed_mapping ] && N=16777216
  timeout -k 10 300 python bench.py --workload $W --candidates $N --no-stream --no-eval --no-cpu-baseline > gpurun_out/${T}_b_$W.json 2> gpurun_out/${T}_b_$W.err || { tail -20 gpurun_out/${T}_b_$W.err; exit 1; }
  cat gpurun_out/${T}_b_$W.json >> gpurun_out/${T}_workloads.jsonl
done
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
# A/B: small dictionaries as gathers (the round-2 emission)
for W in token_transfer_underflow suicide_kill; do
  MYTHGPU_JIT_SELECT_DICT=0 timeout -k 10 300 python bench.py --workload $W --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/${T}_b_${W}_gather.json 2> gpurun_out/${T}_b_${W}_gather.err || { tail -20 gpurun_out/${T}_b_${W}_gather.err; exit 1; }
  cat gpurun_out/${T}_b_${W}_gather.json >> gpurun_out/${T}_workloads.jsonl
done
