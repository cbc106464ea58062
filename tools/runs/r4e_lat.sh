set -o pipefail
mkdir -p gpurun_out
MYTHGPU_JIT_TIMING=1 timeout -k 10 200 python tools/asm_latency.py > gpurun_out/r4e_asm_latency.jsonl 2> gpurun_out/r4e_asm_latency.err || { tail -20 gpurun_out/r4e_asm_latency.err; exit 1; }
cat gpurun_out/r4e_asm_latency.jsonl
grep "worker (asm)\|jit asm:" gpurun_out/r4e_asm_latency.err | tail -12
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
