#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes (one pass per counter group) of bench.py.
# Usage (on the GPU box): tools/profile.sh [workload] [engine jit|interp] [candidates]
#   -> gpurun_out/prof_<workload>[_interp]/...
#   summary: gpurun_out/prof_<workload>/pmc_<workload>.json (copy to profiles/<tag>_pmc_<workload>.json;
#   bench.py matches it to the kernel by the JIT source SHA it records)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=${1:-token_transfer_underflow}
E=${2:-jit}
N=${3:-268435456}
if [ "$E" = "jit" ]; then D=gpurun_out/prof_$W; K=mgj_search; elif [ "$E" = "asm" ]; then D=gpurun_out/prof_${W}_asm; K=mgj_search; else D=gpurun_out/prof_${W}_$E; K=k_run; fi
rm -rf $D && mkdir -p $D
B="python3 bench.py --workload $W --engine $E --candidates $N --no-cpu-baseline --no-ttfm --no-stream --no-eval"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $B --steps 10 --warmup 2 > $D/trace.log 2>&1 || exit $?
grep "^{\"metric\"" $D/trace.log > $D/bench_under_trace.json
pass=0
for counters in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
                "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"; do
  pass=$((pass+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters -d $D/pmc$pass -o run --output-format csv -- $B --steps 2 --warmup 1 > $D/pmc$pass.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $D $W $K > $D/pmc_$W.json
