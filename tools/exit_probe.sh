#!/bin/bash
# GPU box: the exit probe (tools/exit_probe.py) once per configuration, each its own step with its
# own time limit; stops at the first step that does not exit 0 (an abort is the finding).
#   -> gpurun_out/exit_probe.jsonl (one line per step: config, rc, stdout, stderr tail)
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/exit_probe.jsonl
: > $OUT
step() {
  local name="$1"; shift
  env "$@" timeout -k 10 120 python tools/exit_probe.py $PROBE_ARGS > gpurun_out/ep_$name.out 2> gpurun_out/ep_$name.err
  local rc=$?
  python - "$name" "$rc" "$*" <<'PY' >> $OUT
import json, sys
name, rc, envs = sys.argv[1], int(sys.argv[2]), sys.argv[3]
out = open(f"gpurun_out/ep_{name}.out").read()
err = open(f"gpurun_out/ep_{name}.err").read()
print(json.dumps({"step": name, "env": envs, "args": __import__("os").environ.get("PROBE_ARGS", ""), "rc": rc,
                  "stdout": out.strip()[-400:], "stderr_tail": err.strip()[-1500:]}))
PY
  cat $OUT | tail -1
  return $rc
}
# 1. round 2's configuration: compiler in-process, skip-uniform on, Python atexit handler removed
PROBE_ARGS=--no-atexit step inproc_skipuniform_noatexit MYTHGPU_JIT_ISOLATE=0 MYTHGPU_JIT_SKIP_UNIFORM=1 && \
# 2. the same with the atexit handler (round 2's shipped fix)
PROBE_ARGS= step inproc_skipuniform_atexit MYTHGPU_JIT_ISOLATE=0 MYTHGPU_JIT_SKIP_UNIFORM=1 && \
# 3. this round's default: the compiler in its own process, no atexit handler
PROBE_ARGS=--no-atexit step helper_noatexit MYTHGPU_JIT_SKIP_UNIFORM=1 && \
PROBE_ARGS= step helper_default MYTHGPU_JIT_ISOLATE=1
