set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "edge or narrow or sha3 or division or sdiv or keccak or workload or random or vmtest or exp" > gpurun_out/dv_pytest.log 2>&1 || { tail -30 gpurun_out/dv_pytest.log; exit 1; }
tail -2 gpurun_out/dv_pytest.log
bash tools/profile.sh sha3_keyed_mapping jit 16777216 && bash tools/profile.sh sha3_keyed_mapping interp 1048576
