# round 4, run FIN4: the whole GPU suite and smoke at HEAD (after the first tier's Bool lookups)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4fin4_pytest.log 2>&1 || { tail -40 gpurun_out/r4fin4_pytest.log; exit 1; }
tail -3 gpurun_out/r4fin4_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fin4_smoke.log 2>&1 || { tail -20 gpurun_out/r4fin4_smoke.log; exit 1; }
tail -3 gpurun_out/r4fin4_smoke.log
