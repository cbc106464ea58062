"""The eval kernels' HBM rate against the SoA shape (GPU box): for each workload and kernel (O3 /
first tier) the candidate count n -- a power of two puts every coordinate row 2^k bytes after the
last, a padded n does not -- and, for the first tier, the row queue depth (MYTHGPU_JIT_ASM_PREFETCH
in a child process).  One JSON line per point:  python tools/eval_sweep.py > gpurun_out/eval_sweep.jsonl"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CHILD = r"""
import json, sys
sys.path.insert(0, %r)
import torch
import bench
from mythril_amd import native
torch.cuda.set_device(0)
eng = native.Engine.get()
w, n, asm = sys.argv[1], int(sys.argv[2]), sys.argv[3] == "1"
r = bench.eval_roofline(eng, torch, w, n, "/nonexistent", reps=5, asm=asm)
print(json.dumps({"workload": w, "n": n, "asm": asm, "prefetch": __import__("os").environ.get("MYTHGPU_JIT_ASM_PREFETCH"),
                  "kernel_ms": round(r["kernel_ms"], 4), "rows": r["soa_rows_read"], "hbm_frac": round(r["hbm"]["frac"], 4)}))
""" % str(ROOT)

points = []
for w in ("token_transfer_underflow", "walletlibrary_kill"):
    for n in (1 << 22, (1 << 22) + 64 * 67, 1 << 23, (1 << 23) + 64 * 67):
        points.append((w, n, "0", None))
        points.append((w, n, "1", None))
    for d in ("8", "16", "32"):
        points.append((w, (1 << 22) + 64 * 67, "1", d))
for w, n, asm, d in points:
    env = dict(os.environ)
    if d:
        env["MYTHGPU_JIT_ASM_PREFETCH"] = d
    r = subprocess.run([sys.executable, "-c", CHILD, w, str(n), asm], capture_output=True, text=True, env=env, timeout=120)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps({"workload": w, "n": n, "asm": asm, "error": r.stderr[-300:]})
    print(line, flush=True)
