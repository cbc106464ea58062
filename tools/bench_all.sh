#!/bin/bash
# Every workload: PMC + kernel-trace profile of its JIT kernel, then bench.py (which reads the
# profile back for roofline.frac).  -> gpurun_out/bench_all.jsonl, gpurun_out/prof_<w>/
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_all.jsonl
for W in ${@:-suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill sha3_keyed_mapping}; do
  N=268435456; [ "$W" = sha3_keyed_mapping ] && N=16777216
  bash tools/profile.sh $W jit $N || exit 1
  cp gpurun_out/prof_$W/pmc_$W.json gpurun_out/pmc_$W.json
  timeout -k 10 300 python bench.py --workload $W --candidates $N --pmc-dir gpurun_out --no-stream --no-eval > gpurun_out/b_$W.json 2> gpurun_out/b_$W.err || { tail -5 gpurun_out/b_$W.err; exit 1; }
  cat gpurun_out/b_$W.json >> gpurun_out/bench_all.jsonl
done
