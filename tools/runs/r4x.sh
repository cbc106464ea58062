# round 4, run X: first tier with UMUL_NOOVF (C3 inside): parity, C3 rate on the tier, C3 hard-ish TTFM
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_asm.py -x -q --timeout 200 --timeout-method thread -k "not eval_workload" > gpurun_out/r4x_pytest.log 2>&1 || { tail -30 gpurun_out/r4x_pytest.log; exit 1; }
tail -2 gpurun_out/r4x_pytest.log
timeout -k 10 200 python bench.py --workload bectoken_batch_overflow --engine asm --candidates 268435456 --no-cpu-baseline --no-ttfm --no-stream --no-eval > gpurun_out/r4x_a.json 2> gpurun_out/r4x_a.err || { tail -5 gpurun_out/r4x_a.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4x_a.json')); print('C3 first tier', d['value'], d['roofline'].get('kernel_ms'))"
