#!/bin/bash
# GPU box: PMC + kernel-trace profile of every workload's JIT search kernel and the bench line that
# reads it back (roofline.frac), then an A/B of JIT compiler options.
#   tools/r3_prof.sh <tag> [workloads...]  -> gpurun_out/<tag>_prof.jsonl, gpurun_out/prof_<w>/
set -o pipefail
T=${1:-r3p}; shift
mkdir -p gpurun_out
: > gpurun_out/${T}_prof.jsonl
for W in ${@:-suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill sha3_keyed_mapping}; do
  N=268435456; [ "$W" = sha3_keyed_mapping ] && N=16777216
  bash tools/profile.sh $W jit $N || exit 1
  cp gpurun_out/prof_$W/pmc_$W.json gpurun_out/pmc_$W.json
  timeout -k 10 300 python bench.py --workload $W --candidates $N --pmc-dir gpurun_out --no-stream --no-eval --no-cpu-baseline > gpurun_out/${T}_b_$W.json 2> gpurun_out/${T}_b_$W.err || { tail -5 gpurun_out/${T}_b_$W.err; exit 1; }
  cat gpurun_out/${T}_b_$W.json >> gpurun_out/${T}_prof.jsonl
done
