set -o pipefail
bash tools/profile_eval.sh token_transfer_underflow 4194304 && bash tools/profile_eval.sh walletlibrary_kill 4194304 && ls gpurun_out/prof_eval_*/
