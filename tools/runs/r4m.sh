# round 4, run M: where the hard query's cold first-tier compile spends its time (worker stage timing)
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python bench.py --gpus 1 --no-cpu-baseline --no-eval --no-stream > gpurun_out/r4m_bench$k.json 2> gpurun_out/r4m_bench$k.err || { tail -20 gpurun_out/r4m_bench$k.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r4m_bench$k.json')); h=d['time_to_first_model_hard']; print('hard', h['cold_ms'], h['cold_engine'], h['cold_timing'])"
grep -n "jit\|comgr\|warm" gpurun_out/r4m_bench$k.err | tail -40
done
