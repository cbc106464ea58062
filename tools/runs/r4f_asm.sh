# round 4, run F: first tier with LDS dictionaries: parity, rate, PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_asm.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1 || { tail -30 gpurun_out/r4f_pytest.log; exit 1; }
tail -2 gpurun_out/r4f_pytest.log
timeout -k 10 120 python tools/launch_size.py token_transfer_underflow --asm > gpurun_out/r4f_launch_size_asm.jsonl || exit 1
cat gpurun_out/r4f_launch_size_asm.jsonl
bash tools/profile.sh token_transfer_underflow asm 268435456 || exit 1
cp gpurun_out/prof_token_transfer_underflow_asm/pmc_token_transfer_underflow.json gpurun_out/pmc_asm_token_transfer_underflow.json
python3 -c "import json; d=json.load(open('gpurun_out/pmc_asm_token_transfer_underflow.json')); c=d['per_launch_counters']; print(json.dumps(d.get('derived'))); print('wait', c['SQ_WAIT_ANY']/c['SQ_WAVE_CYCLES'], 'vmem/group', c['SQ_INSTS_VMEM_RD']/(268435456/64), 'lds/group', c['SQ_INSTS_LDS']/(268435456/64))"
