set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "sweep or jit or isolation" > gpurun_out/r3e_pytest.log 2>&1 || { tail -30 gpurun_out/r3e_pytest.log; exit 1; }
tail -2 gpurun_out/r3e_pytest.log
bash tools/bench_all.sh suicide_kill token_transfer_underflow bectoken_batch_overflow || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err || { tail -20 gpurun_out/r3e_bench.err; exit 1; }
cat gpurun_out/r3e_bench.json
