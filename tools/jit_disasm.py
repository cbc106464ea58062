"""Host-only: emit + hipRTC-compile the search kernel of a workload and count its
instructions (static, per loop iteration of the straight-line body) — a CPU-side
proxy for the PMC SQ_INSTS_VALU count while iterating on the code generator.

usage: python tools/jit_disasm.py [workload ...]   (writes /tmp/jd/<workload>.{hip,co,s})
"""
import collections
import os
import re
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from mythril_amd import native, search, ssa, workloads  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def main():
    names = sys.argv[1:] or ["token_transfer_underflow"]
    out = Path("/tmp/jd")
    out.mkdir(exist_ok=True)
    for name in names:
        roots = [c.raw for c in workloads.WORKLOADS[name]()]
        P = search.FLATTEN_CACHE.flatten(roots)
        blob = search.default_generator(P, roots=roots).blob()
        os.environ["MYTHGPU_JIT_DUMP"] = str(out / name)
        t = time.perf_counter()
        native.jit_source(P.to_bytes(), blob, compile=True)
        ms = (time.perf_counter() - t) * 1e3
        asm = subprocess.run([OBJDUMP, "-d", str(out / f"{name}.co")], capture_output=True, text=True).stdout
        (out / f"{name}.s").write_text(asm)
        ops = re.findall(r"^\s+([vs]_[a-z0-9_]+)", asm, re.M)
        cnt = collections.Counter(ops)
        valu = sum(v for k, v in cnt.items() if k.startswith("v_"))
        salu = sum(v for k, v in cnt.items() if k.startswith("s_") and k != "s_nop")
        print(f"{name}: coords={len(P.coords)} nodes={len(P.nodes)} compile={ms:.0f} ms  static VALU={valu} "
              f"SALU={salu} s_nop={cnt['s_nop']}  top: " +
              ", ".join(f"{k}={v}" for k, v in cnt.most_common(8)))


if __name__ == "__main__":
    main()
