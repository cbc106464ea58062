# round 5, run F: first-tier small-dictionary LDS reads + deferred LDS waits + two assembly helpers +
# products as v_mad_u64_u32 (and without: MYTHGPU_JIT_ASM_NO_MAD=1) —
# asm suite, tier rates, C5's hard query cold; then two diagnostics: the first tier on C1 with its
# dictionaries gathered from global memory (MYTHGPU_JIT_ASM_NO_LDS=1), and the O3 headline kernel with
# conflict-free dictionary reads (MYTHGPU_JIT_DICT_SPREAD=1, wrong verdicts: what LDS bank conflicts cost)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_jit.py -m gpu -x -q --durations=12 --timeout 300 --timeout-method thread > gpurun_out/r5f_pytest.log 2>&1 || { tail -40 gpurun_out/r5f_pytest.log; exit 1; }
tail -2 gpurun_out/r5f_pytest.log
: > gpurun_out/r5f_rates.jsonl
rate() {  # workload engine candidates tag [env...]
  local w=$1 e=$2 n=$3 tag=$4; shift 4
  env "$@" timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5f_b.json 2> gpurun_out/r5f_b.err || { tail -20 gpurun_out/r5f_b.err; return 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/r5f_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'tag': '$tag', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5f_rates.jsonl
}
for w in token_transfer_underflow walletlibrary_kill suicide_kill bectoken_batch_overflow etherstore_reentrancy; do
  rate $w asm 268435456 default || exit 1
done
rate sha3_keyed_mapping asm 16777216 default || exit 1
rate bectoken_batch_overflow asm 268435456 no_lds MYTHGPU_JIT_ASM_NO_LDS=1 || exit 1
rate bectoken_batch_overflow asm 268435456 no_mad MYTHGPU_JIT_ASM_NO_MAD=1 || exit 1
rate sha3_keyed_mapping asm 16777216 no_mad MYTHGPU_JIT_ASM_NO_MAD=1 || exit 1
rate token_transfer_underflow jit 1073741824 default || exit 1
rate token_transfer_underflow jit 1073741824 dict_spread MYTHGPU_JIT_DICT_SPREAD=1 || exit 1
cat gpurun_out/r5f_rates.jsonl
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python bench.py --workload sha3_keyed_mapping --candidates 16777216 --steps 3 --no-stream --no-eval --no-cpu-baseline > gpurun_out/r5f_bench_c5.json 2> gpurun_out/r5f_bench_c5.err || { tail -20 gpurun_out/r5f_bench_c5.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5f_bench_c5.json").read().strip().splitlines()[-1])
h = d.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine", "index", "candidates")}), json.dumps(h.get("cold_timing")))
PY
grep -i "jit worker" gpurun_out/r5f_bench_c5.err | head -8
