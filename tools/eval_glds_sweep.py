"""The first tier's tiled eval kernel against its row queue (GPU box): the register queue
(MYTHGPU_JIT_ASM_GLDS=0), the LDS-staged queue at the depth the compiler picks (default) and at fixed
depths, and with the greedy constraint order.  One JSON line per point:
  python tools/eval_glds_sweep.py > gpurun_out/eval_glds.jsonl"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CHILD = r"""
import json, os, sys
sys.path.insert(0, %r)
import torch
import bench
from mythril_amd import native
torch.cuda.set_device(0)
eng = native.Engine.get()
w, n = sys.argv[1], int(sys.argv[2])
r = bench.eval_roofline(eng, torch, w, n, "/nonexistent", reps=5, asm=True, tiled=True)
print(json.dumps({"workload": w, "n": n, "glds": os.environ.get("MYTHGPU_JIT_ASM_GLDS", "auto"),
                  "greedy": os.environ.get("MYTHGPU_JIT_ASM_GREEDY") == "1",
                  "kernel_ms": round(r["kernel_ms"], 4), "rows": r["soa_rows_read"],
                  "hbm_frac": round(r["hbm"]["frac"], 4), "sha": r.get("jit_source_sha16")}))
""" % str(ROOT)

points = []
for w in ("walletlibrary_kill", "token_transfer_underflow"):
    for g in (None, "0", "12", "20", "32"):
        points.append((w, g, None))
    points.append((w, None, "1"))  # the greedy constraint order (MYTHGPU_JIT_ASM_GREEDY=1)
for w, g, ng in points:
    env = dict(os.environ)
    if g:
        env["MYTHGPU_JIT_ASM_GLDS"] = g
    if ng:
        env["MYTHGPU_JIT_ASM_GREEDY"] = ng
    r = subprocess.run([sys.executable, "-c", CHILD, w, str(1 << 22)], capture_output=True, text=True, env=env,
                       timeout=120)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps(
        {"workload": w, "glds": g, "error": r.stderr[-400:]})
    print(line, flush=True)
