# round 4, run K: TLB counters of the eval kernels (C2 vs C4; is the 243-row C4 stream translation-bound?)
set -o pipefail
mkdir -p gpurun_out/r4k
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/r4k/avail.txt 2>&1 || true
grep -o "TCP_UTCL[A-Z0-9_]*\|TCP_TCP_TA[A-Z_]*\|UTCL2[A-Z0-9_]*\|TCP_PENDING[A-Z_]*\|TCP_TA_TCP_STATE_READ\|TCP_GATE_EN[0-9]\|TCP_TCR_TCP_STALL_CYCLES\|TCP_READ_TAGCONFLICT_STALL_CYCLES\|TCP_TCC_READ_REQ_LATENCY[A-Z_]*" gpurun_out/r4k/avail.txt | sort -u > gpurun_out/r4k/tcp_names.txt || true
cat gpurun_out/r4k/tcp_names.txt
for W in token_transfer_underflow walletlibrary_kill; do
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCR_TCP_STALL_CYCLES_sum -d gpurun_out/r4k/$W -o run --output-format csv -- python3 tools/eval_probe.py $W 4194304 2 > gpurun_out/r4k/$W.log 2>&1 || { tail -5 gpurun_out/r4k/$W.log; exit 1; }
done
echo done
