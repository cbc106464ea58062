set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err || { tail -20 gpurun_out/r3d_bench.err; exit 1; }
cat gpurun_out/r3d_bench.json
bash tools/profile_eval.sh token_transfer_underflow || exit 1
bash tools/profile_eval.sh walletlibrary_kill || exit 1
for W in suicide_kill token_transfer_underflow bectoken_batch_overflow walletlibrary_kill sha3_keyed_mapping; do
  bash tools/jit_sweep.sh $W skipu=MYTHGPU_JIT_SKIP_UNIFORM=1 || exit 1
done
