#!/bin/bash
# GPU box: the headline bench line (profiles/ PMC matched), the distributed code path at one
# rank under torch.distributed.run, and the 200 ms LASER-shaped get_model stream over C1-C4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/fc_bench.json 2> gpurun_out/fc_bench.err || { tail -20 gpurun_out/fc_bench.err; exit 1; }
cat gpurun_out/fc_bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/fc_torchrun1.json 2> gpurun_out/fc_torchrun1.err || { tail -20 gpurun_out/fc_torchrun1.err; exit 1; }
cat gpurun_out/fc_torchrun1.json
timeout -k 10 400 python tools/stream_bench.py --budget-ms 200 --workloads suicide_kill,token_transfer_underflow,etherstore_reentrancy,bectoken_batch_overflow,walletlibrary_kill > gpurun_out/fc_stream.jsonl 2> gpurun_out/fc_stream.err || { tail -20 gpurun_out/fc_stream.err; exit 1; }
grep -v '"q"' gpurun_out/fc_stream.jsonl
