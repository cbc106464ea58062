# round 4: the first tier's generator share (PMC, gen-only vs full) against the O3 kernel's, C2 and C4 at 2^28
set -o pipefail
mkdir -p gpurun_out
for W in token_transfer_underflow walletlibrary_kill; do
  MYTHGPU_JIT_ASM_GEN_ONLY=1 bash tools/profile.sh $W asm 268435456 || exit 1
  cp gpurun_out/prof_${W}_asm/pmc_$W.json gpurun_out/pmc_asm_genonly_$W.json
  MYTHGPU_JIT_GEN_ONLY=1 bash tools/profile.sh $W jit 268435456 || exit 1
  cp gpurun_out/prof_$W/pmc_$W.json gpurun_out/pmc_o3_genonly_$W.json
  bash tools/profile.sh $W asm 268435456 || exit 1
  cp gpurun_out/prof_${W}_asm/pmc_$W.json gpurun_out/pmc_asm_full_$W.json
done
for f in gpurun_out/pmc_*_genonly_*.json gpurun_out/pmc_asm_full_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['derived']['valu_wave_instructions_per_candidate'],1), round(d['derived']['salu_instructions_per_candidate'],1))"; done
