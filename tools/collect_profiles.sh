#!/bin/bash
# Copy a tools/bench_all.sh / tools/profile.sh run (gpurun_out/) into profiles/ under a round tag:
#   tools/collect_profiles.sh r02 [workload ...]
set -o pipefail
T=${1:?tag}; shift
for W in ${@:-suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill sha3_keyed_mapping}; do
  D=gpurun_out/prof_$W
  [ -f $D/pmc_$W.json ] || continue
  cp $D/pmc_$W.json profiles/${T}_pmc_$W.json
  cp $D/trace/run_kernel_stats.csv profiles/${T}_rocprof_kernel_stats_$W.csv
done
[ -f gpurun_out/bench_all.jsonl ] && cp gpurun_out/bench_all.jsonl profiles/${T}_bench_workloads.jsonl
exit 0
