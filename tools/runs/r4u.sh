# round 4, run U: a cold easy query's time split
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/cold_probe.py > gpurun_out/r4u_cold.jsonl 2> gpurun_out/r4u_cold.err || { tail -10 gpurun_out/r4u_cold.err; exit 1; }
cat gpurun_out/r4u_cold.jsonl
