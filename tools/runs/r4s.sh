# round 4, run S: the C2 model-verification failure of r4r: which engine / index, with and without the first tier
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/dbg_model.py > gpurun_out/r4s_dbg.jsonl 2> gpurun_out/r4s_dbg.err || { tail -20 gpurun_out/r4s_dbg.err; exit 1; }
cat gpurun_out/r4s_dbg.jsonl
MYTHGPU_JIT_ASM=0 timeout -k 10 200 python tools/dbg_model.py > gpurun_out/r4s_dbg_noasm.jsonl 2>> gpurun_out/r4s_dbg.err || { tail -20 gpurun_out/r4s_dbg.err; exit 1; }
cat gpurun_out/r4s_dbg_noasm.jsonl
