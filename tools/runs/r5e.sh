# round 5, run E: the first tier after the cache soft limit / partial MIXED generation / bitop3
# equality / lookup runs / mask spills — asm + jit + parity suites, rates on both compiled tiers
# (10 steps at 2^28, C5 at 2^24), C5's hard query cold with the queue wait printed, then the first
# tier's PMC passes on C2 and C4 (tools/profile.sh, asm engine)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_asm.py tests/test_gpu_jit.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5e_pytest.log 2>&1 || { tail -40 gpurun_out/r5e_pytest.log; exit 1; }
tail -2 gpurun_out/r5e_pytest.log
: > gpurun_out/r5e_rates.jsonl
for w in token_transfer_underflow walletlibrary_kill suicide_kill bectoken_batch_overflow etherstore_reentrancy sha3_keyed_mapping; do
  n=268435456; [ $w = sha3_keyed_mapping ] && n=16777216
  for e in asm jit; do
    timeout -k 10 200 python bench.py --workload $w --engine $e --candidates $n --steps 10 --warmup 2 --no-stream --no-eval --no-cpu-baseline --no-ttfm > gpurun_out/r5e_b.json 2> gpurun_out/r5e_b.err || { tail -20 gpurun_out/r5e_b.err; exit 1; }
    python -c "
import json; d = json.loads(open('gpurun_out/r5e_b.json').read().strip().splitlines()[-1])
print(json.dumps({'workload': '$w', 'engine': '$e', 'candidates_per_s': d['value'], 'ms_per_step': d['ms_per_step'], 'jit_source_sha16': d['config'].get('jit_source_sha16')}))" >> gpurun_out/r5e_rates.jsonl
  done
done
cat gpurun_out/r5e_rates.jsonl
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python bench.py --workload sha3_keyed_mapping --candidates 16777216 --steps 3 --no-stream --no-eval --no-cpu-baseline > gpurun_out/r5e_bench_c5.json 2> gpurun_out/r5e_bench_c5.err || { tail -20 gpurun_out/r5e_bench_c5.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5e_bench_c5.json").read().strip().splitlines()[-1])
print(json.dumps(d.get("jit_asm_tier")))
h = d.get("time_to_first_model_hard") or {}
print(json.dumps({k: h.get(k) for k in ("cold_ms", "warm_ms", "cold_engine", "index", "candidates")}), json.dumps(h.get("cold_timing")))
PY
grep -i "jit worker" gpurun_out/r5e_bench_c5.err | head -6
timeout -k 10 600 bash tools/profile.sh token_transfer_underflow asm && timeout -k 10 600 bash tools/profile.sh walletlibrary_kill asm && ls gpurun_out/prof_token_transfer_underflow_asm gpurun_out/prof_walletlibrary_kill_asm
