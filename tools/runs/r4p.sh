# round 4, run P: headline PMC at HEAD's O3 source (bench frac), eval kernels' PMC (O3 row-major, first tier tiled)
set -o pipefail
mkdir -p gpurun_out
bash tools/profile.sh token_transfer_underflow jit 1073741824 || { echo "profile headline failed"; exit 1; }
cat gpurun_out/prof_token_transfer_underflow/pmc_token_transfer_underflow.json | head -c 600; echo
for W in token_transfer_underflow walletlibrary_kill; do
  bash tools/profile_eval.sh $W 4194304 0 0 || { echo "profile eval $W failed"; exit 1; }
  bash tools/profile_eval.sh $W 4194304 1 1 || { echo "profile evalasm tiled $W failed"; exit 1; }
done
ls gpurun_out/prof_*/pmc_*.json
