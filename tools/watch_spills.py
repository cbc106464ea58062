"""SGPR spill traffic of the watch-row eval kernels (host-only): v_readlane / v_writelane in the code
object of each workload's unspecialised program WITH its model watch rows — the O3 kernel (indexed
rows, and walking rows with MYTHGPU_JIT_WATCH_WALK=1 in a child) and the first tier's (jit_asm.cpp).

  python tools/watch_spills.py > profiles/rNN_watch_spills.jsonl"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CHILD = r"""
import collections, json, os, re, subprocess, sys
sys.path.insert(0, %r)
from mythril_amd import native, search, workloads
name, tier, dump = sys.argv[1], sys.argv[2], sys.argv[3]
P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
os.environ["MYTHGPU_JIT_DUMP"] = dump
if tier == "asm":
    src = native.jit_asm(P.to_bytes(), None, compile=True)
else:
    src = native.jit_source(P.to_bytes(), None, compile=True)
dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", dump + ".co"], capture_output=True, text=True).stdout
ops = collections.Counter(re.findall(r"^\s+([vs]_[a-z0-9_]+)", dis, re.M))
vg = re.findall(r"vgpr_count:\s+(\d+)", subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", dump + ".co"], capture_output=True, text=True).stdout)
print(json.dumps({"workload": name, "kernel": tier, "watch_words": P.watch_words if hasattr(P, "watch_words") else None,
                  "v_readlane": ops["v_readlane_b32"], "v_writelane": ops["v_writelane_b32"],
                  "static_valu": sum(v for k, v in ops.items() if k.startswith("v_")), "vgpr_count": vg[:1]}))
""" % str(ROOT)


def main():
    names = sys.argv[1:] or ["walletlibrary_kill", "token_transfer_underflow"]
    for name in names:
        for tier, env in (("o3", {}), ("o3-walk", {"MYTHGPU_JIT_WATCH_WALK": "1"}), ("asm", {})):
            with tempfile.TemporaryDirectory() as d:
                e = dict(os.environ, MYTHGPU_JIT_ISOLATE="0", MYTHGPU_JIT_DISK_CACHE="0", **env)
                r = subprocess.run([sys.executable, "-c", CHILD, name, "asm" if tier == "asm" else "o3", d + "/k"],
                                   capture_output=True, text=True, env=e)
                line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps({"error": r.stderr[-300:]})
                rec = json.loads(line)
                rec["kernel"] = tier
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
