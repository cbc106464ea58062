# round 4, run V: kernels warmed at mg_init -- cold easy query split again, parity subset, smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/cold_probe.py > gpurun_out/r4v_cold.jsonl 2> gpurun_out/r4v_cold.err || { tail -10 gpurun_out/r4v_cold.err; exit 1; }
cat gpurun_out/r4v_cold.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capture.py tests/test_gpu_multidevice.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4v_pytest.log 2>&1 || { tail -30 gpurun_out/r4v_pytest.log; exit 1; }
tail -2 gpurun_out/r4v_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
