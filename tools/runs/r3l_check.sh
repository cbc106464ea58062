set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/config_sweeps.py > gpurun_out/r3l_sweeps.jsonl 2> gpurun_out/r3l_sweeps.err || { tail -20 gpurun_out/r3l_sweeps.err; exit 1; }
cat gpurun_out/r3l_sweeps.jsonl
: > gpurun_out/r3l_eval_ab.jsonl
for W in token_transfer_underflow walletlibrary_kill; do
  for V in "" 2 3 4; do
    MYTHGPU_JIT_WAVES=$V timeout -k 10 120 python tools/eval_probe.py $W 4194304 5 > gpurun_out/r3l_e.json 2> gpurun_out/r3l_e.err || { tail -5 gpurun_out/r3l_e.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r3l_e.json').read().splitlines()[-1]); print(json.dumps({'workload':'$W','waves':'$V','kernel_ms':d['roofline']['kernel_ms'],'hbm_frac':d['eval']['hbm']['frac']}))" >> gpurun_out/r3l_eval_ab.jsonl
  done
done
cat gpurun_out/r3l_eval_ab.jsonl
bash tools/profile_eval.sh token_transfer_underflow && bash tools/profile_eval.sh walletlibrary_kill || exit 1
bash tools/profile.sh token_transfer_underflow interp 4194304 || exit 1
