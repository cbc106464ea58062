# round 4, run FIN3 (HEAD after the forced and ITE compare pushdown; as FIN2, plus the C4 row; after the
# tier's compare-difference cache): headline + eval PMC at HEAD's sources (copied into profiles/ on
# the box so the bench line matches them), the whole GPU suite, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out
bash tools/profile.sh token_transfer_underflow jit 1073741824 || { echo "profile headline failed"; exit 1; }
cp gpurun_out/prof_token_transfer_underflow/pmc_token_transfer_underflow.json profiles/r04f3_pmc_headline_token_transfer_underflow.json
for W in token_transfer_underflow walletlibrary_kill; do
  bash tools/profile_eval.sh $W 4194304 0 0 || { echo "profile eval $W failed"; exit 1; }
  cp gpurun_out/prof_eval_$W/pmc_eval_$W.json profiles/r04f3_pmc_eval_$W.json
  bash tools/profile_eval.sh $W 4194304 1 1 || { echo "profile evalasm tiled $W failed"; exit 1; }
  cp gpurun_out/prof_evalasm_tiled_$W/pmc_evalasm_tiled_$W.json profiles/r04f3_pmc_evalasm_tiled_$W.json
done
bash tools/profile.sh walletlibrary_kill jit 268435456 || { echo "profile C4 failed"; exit 1; }
cp gpurun_out/prof_walletlibrary_kill/pmc_walletlibrary_kill.json profiles/r04f3_pmc_walletlibrary_kill.json
cp gpurun_out/prof_walletlibrary_kill/trace/run_kernel_stats.csv profiles/r04f3_rocprof_kernel_stats_walletlibrary_kill.csv
timeout -k 10 300 python bench.py --workload walletlibrary_kill --candidates 268435456 --no-stream --no-eval > profiles/r04f3_bench_walletlibrary_kill.json 2> gpurun_out/r4fin3_c4.err || { tail -5 gpurun_out/r4fin3_c4.err; exit 1; }
mkdir -p gpurun_out/f3 && cp profiles/r04f3_* gpurun_out/f3/
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r4fin3_pytest.log 2>&1 || { tail -40 gpurun_out/r4fin3_pytest.log; exit 1; }
tail -20 gpurun_out/r4fin3_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fin3_smoke.log 2>&1 || { tail -20 gpurun_out/r4fin3_smoke.log; exit 1; }
tail -3 gpurun_out/r4fin3_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r4fin3_bench.json 2> gpurun_out/r4fin3_bench.err || { tail -20 gpurun_out/r4fin3_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r4fin3_bench.json')); print('value', d['value'], 'frac', d['roofline'].get('frac'), 'traffic', d['roofline'].get('traffic'), 'ttfm', d['time_to_first_model_ms'], d['time_to_first_model_cold_ms'], 'hard', d['time_to_first_model_hard']['cold_ms'], d['time_to_first_model_hard']['cold_engine'], 'cpu', d['cpu_baseline']['value'])
for e in d['config'].get('roofline_eval', d.get('roofline_eval', [])) or []: print(json.dumps(e)[:300])"
