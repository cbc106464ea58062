#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes of the eval kernel (mgj_eval, unspecialised program,
# HBM-resident SoA) -- tools/eval_probe.py.  Usage (GPU box): tools/profile_eval.sh [workload] [candidates] [asm 0|1] [tiled 0|1]
#   -> gpurun_out/prof_<tag><workload>/pmc_<tag><workload>.json, tag eval_ / evalasm_ (+ tiled_)
#   (copy to profiles/<round>_pmc_<tag><workload>.json: bench.py matches it by source SHA)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=${1:-token_transfer_underflow}
N=${2:-4194304}
A=${3:-0}
T=${4:-0}
TAG=eval_; [ "$A" = "1" ] && TAG=evalasm_; [ "$T" = "1" ] && TAG=${TAG}tiled_
D=gpurun_out/prof_$TAG$W
rm -rf $D && mkdir -p $D
B="python3 tools/eval_probe.py $W $N"
BA="$A $T"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $B 10 $BA > $D/trace.log 2>&1 || exit $?
grep "^{\"metric\"" $D/trace.log > $D/bench_under_trace.json
pass=0
for counters in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
                "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"; do
  pass=$((pass+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters -d $D/pmc$pass -o run --output-format csv -- $B 2 $BA > $D/pmc$pass.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $D $TAG$W mgj_eval > $D/pmc_$TAG$W.json
