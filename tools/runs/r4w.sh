# round 4, run W: O3 eval kernel occupancy hint (amdgpu_waves_per_eu) on C4, tiled and row-major
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r4w.jsonl
for WV in 0 3 4; do
  for T in 1 0; do
    MYTHGPU_JIT_WAVES=$WV MYTHGPU_JIT_DISK_CACHE=0 timeout -k 10 120 python tools/eval_probe.py walletlibrary_kill 4194304 5 0 $T > gpurun_out/r4w_p.json 2> gpurun_out/r4w_p.err || { tail -5 gpurun_out/r4w_p.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4w_p.json').read().splitlines()[-1])['eval']; print(json.dumps({'waves_per_eu': $WV, 'tiled': $T, 'kernel_ms': round(d['kernel_ms'],4), 'hbm_frac': round(d['hbm']['frac'],4)}))" >> gpurun_out/r4w.jsonl
  done
done
cat gpurun_out/r4w.jsonl
