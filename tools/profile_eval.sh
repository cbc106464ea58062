#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes of the eval kernel (mgj_eval, unspecialised program,
# HBM-resident SoA) -- tools/eval_probe.py.  Usage (GPU box): tools/profile_eval.sh [workload] [candidates]
#   -> gpurun_out/prof_eval_<workload>/pmc_eval_<workload>.json (copy to profiles/<tag>_pmc_eval_<workload>.json)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=${1:-token_transfer_underflow}
N=${2:-4194304}
D=gpurun_out/prof_eval_$W
rm -rf $D && mkdir -p $D
B="python3 tools/eval_probe.py $W $N"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $B 10 > $D/trace.log 2>&1 || exit $?
grep "^{\"metric\"" $D/trace.log > $D/bench_under_trace.json
pass=0
for counters in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
                "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"; do
  pass=$((pass+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters -d $D/pmc$pass -o run --output-format csv -- $B 2 > $D/pmc$pass.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $D eval_$W mgj_eval > $D/pmc_eval_$W.json
