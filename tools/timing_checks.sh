# Wall-clock bounds kept out of the parity run (pytest -m gpu prints these timings only):
# time to first model and the early-stop split launch at four virtual devices vs one.
# Run on a GPU box:  bash tools/timing_checks.sh
set -o pipefail
mkdir -p gpurun_out
MYTHGPU_TIMING_ASSERTS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_multidevice.py -m gpu -x -v -s \
  --timeout 240 --timeout-method thread -k "four_devices or stops_at_first_hit" > gpurun_out/timing_checks.log 2>&1
rc=$?
tail -20 gpurun_out/timing_checks.log
exit $rc
