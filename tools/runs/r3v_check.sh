set -o pipefail
mkdir -p gpurun_out
bash tools/runs/r3_ab.sh r3v "bpc32=" "bpc16=MYTHGPU_JIT_BPC=16" "bpc48=MYTHGPU_JIT_BPC=48" "bpc64=MYTHGPU_JIT_BPC=64" && cat gpurun_out/r3v_ab.jsonl
