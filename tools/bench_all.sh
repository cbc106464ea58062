#!/bin/bash
# Bench every workload on one GPU (one JSON line each) -> gpurun_out/bench_workloads.jsonl
set -o pipefail
out=gpurun_out/bench_workloads.jsonl
: > $out
for w in suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill sha3_keyed_mapping; do
  timeout -k 10 150 python bench.py --workload $w --cpu-seconds ${CPU_SECONDS:-4} > gpurun_out/bench_$w.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$w.log >> $out
done
