# round 4, run B: the JIT's assembly tier against the C port on the GPU; multi-device stop; launch sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_multidevice.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1
rc=$?
tail -45 gpurun_out/r4b_pytest.log
[ $rc -eq 0 ] || exit $rc
for mg in 0 16; do
  MYTHGPU_JIT_MIN_GROUPS=$mg timeout -k 10 120 python tools/launch_size.py token_transfer_underflow >> gpurun_out/r4b_launch_size.jsonl || exit 1
done
timeout -k 10 120 python tools/launch_size.py token_transfer_underflow --asm >> gpurun_out/r4b_launch_size.jsonl || exit 1
cat gpurun_out/r4b_launch_size.jsonl
