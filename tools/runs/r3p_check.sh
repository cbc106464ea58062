set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3p_pytest.log 2>&1 || { tail -30 gpurun_out/r3p_pytest.log; exit 1; }
tail -2 gpurun_out/r3p_pytest.log
: > gpurun_out/r3p_interp_ab.jsonl
for V in "160" "255"; do
  for W in walletlibrary_kill token_transfer_underflow; do
    MYTHGPU_INTERP_LDS_MAX=$V timeout -k 10 120 python bench.py --workload $W --engine interp --candidates 4194304 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r3p_i.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3p_i.json')); print(json.dumps({'engine':'interp','workload':'$W','lds_max':$V,'value':d['value']}))" >> gpurun_out/r3p_interp_ab.jsonl
  done
done
cat gpurun_out/r3p_interp_ab.jsonl
bash tools/runs/r3_ab.sh r3p "base=" && cat gpurun_out/r3p_ab.jsonl
