set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r3ad_ab.jsonl
for V in "bpc64=" "bpc32=MYTHGPU_JIT_BPC=32" "bpc128=MYTHGPU_JIT_BPC=128" "bpc64b="; do
  L=${V%%=*}; E=${V#*=}
  env $E timeout -k 10 300 python bench.py --no-stream --no-eval --no-cpu-baseline --no-ttfm --steps 20 --warmup 5 > gpurun_out/r3ad_b.json 2> gpurun_out/r3ad_b.err || { tail -5 gpurun_out/r3ad_b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r3ad_b.json')); print(json.dumps({'variant':'$L','value':d['value'],'kernel_ms':d['roofline']['kernel_ms'],'ms_per_step':d['ms_per_step']}))" >> gpurun_out/r3ad_ab.jsonl
done
cat gpurun_out/r3ad_ab.jsonl
