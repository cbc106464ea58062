"""Instructions per candidate of the first tier's eval kernel (mgj_eval, tiled SoA, no watch rows: the
kernel bench.py's roofline_eval runs) on the CPU simulator, optionally per program instruction.

  python tools/eval_count.py [workload ...] [K=V ...]     (MYTHGPU_JIT_ASM_ANNOTATE=1: per instruction;
                                                          EVAL_LAYOUT=rowmajor: the [row][candidate] SoA)"""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    from mythril_amd import search, workloads
    from tests.test_asm_sim import _cached, record

    class TPF:
        def mktemp(self, name):
            return Path(tempfile.mkdtemp(prefix=name))

    exe = _cached(TPF(), sanitize=False)
    env = dict(os.environ, ASMSIM_COUNT="1")
    names = []
    for a in sys.argv[1:]:
        if "=" in a:
            k, v = a.split("=", 1)
            env[k] = v
        else:
            names.append(a)
    for name in names or ["token_transfer_underflow", "walletlibrary_kill"]:
        P, _ = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        P.set_watch([])
        kind = 1 if env.get("EVAL_LAYOUT") == "rowmajor" else 2  # record kind 1: row-major SoA, 2: tiled
        r = subprocess.run([str(exe)], input=record(kind, P.to_bytes(), None, 7, 0, 64 * 32), capture_output=True,
                           env=env)
        out = r.stdout.decode()
        tags = []
        for ln in out.splitlines():
            if ln.startswith("count eval:"):
                print(name, ln[len("count eval:"):].strip())
            elif ln.startswith("records=") and " ok=1 " not in ln:
                print(name, "(verdicts DIFFER from the C port)", ln)
            elif ln.startswith("count tag "):
                t, v = ln[len("count tag "):].rsplit(":", 1)
                va, _, sa = v.strip().partition(" salu ")
                tags.append((float(va), float(sa or 0), t.strip()))
        for v, sv, t in sorted(tags, reverse=True)[:int(env.get("ASMSIM_TOP", "30"))]:
            print(f"  {v:8.2f} {sv:8.2f}  {t}")


if __name__ == "__main__":
    main()
