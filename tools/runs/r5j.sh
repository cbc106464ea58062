# round 5, run J: where the VMTests read-back replay's time goes (per phase, default tier vs O3)
set -o pipefail
mkdir -p gpurun_out
MYTHGPU_JIT_TIMING=1 timeout -k 10 300 python tools/vmtests_timing.py 40 > gpurun_out/r5j_vmt.json 2> gpurun_out/r5j_vmt.err || { tail -20 gpurun_out/r5j_vmt.err; exit 1; }
cat gpurun_out/r5j_vmt.json
grep "jit worker" gpurun_out/r5j_vmt.err | head -30
