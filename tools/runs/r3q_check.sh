set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3q_pytest.log 2>&1 || { tail -30 gpurun_out/r3q_pytest.log; exit 1; }
tail -2 gpurun_out/r3q_pytest.log
timeout -k 10 200 python tools/interp_latency.py > gpurun_out/r3q_interp_latency.jsonl 2>&1 || exit 1
: > gpurun_out/r3q_interp_ab.jsonl
for W in suicide_kill token_transfer_underflow etherstore_reentrancy bectoken_batch_overflow walletlibrary_kill sha3_keyed_mapping; do
  for N in 1 0; do
    MYTHGPU_INTERP_SINK=$N timeout -k 10 120 python bench.py --workload $W --engine interp --candidates 4194304 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r3q_i.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3q_i.json')); print(json.dumps({'engine':'interp','workload':'$W','sink':$N,'value':d['value']}))" >> gpurun_out/r3q_interp_ab.jsonl
  done
done
cat gpurun_out/r3q_interp_ab.jsonl
timeout -k 10 400 python bench.py --pmc-dir gpurun_out --no-cpu-baseline > gpurun_out/r3q_bench.json 2> gpurun_out/r3q_bench.err || { tail -20 gpurun_out/r3q_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3q_bench.json')); print(d['value'], d['time_to_first_model_ms'], d['time_to_first_model_cold_ms'], json.dumps(d['time_to_first_model_hard']))"
