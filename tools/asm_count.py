"""Instructions per candidate of the first tier's search kernel on the CPU simulator (tests/asmsim):
every workload, a full-evaluation launch (no early exit) over a window of 64-candidate groups, VALU
and SALU lane-instructions per candidate (the PMC's SQ_INSTS_VALU x 64 / candidates, without a GPU).

  python tools/asm_count.py [workload ...] [--env K=V ...]"""
import os
import random
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    from mythril_amd import search, workloads
    from tests.test_asm_sim import _cached, record
    import pytest  # noqa: F401  (the builder's skip path)

    class TPF:  # the fixture's tmp_path_factory, outside pytest
        def mktemp(self, name):
            import tempfile
            return Path(tempfile.mkdtemp(prefix=name))

    names = [a for a in sys.argv[1:] if "=" not in a] or sorted(workloads.WORKLOADS)
    env = dict(os.environ, ASMSIM_COUNT="1")
    for a in sys.argv[1:]:
        if "=" in a:
            k, v = a.split("=", 1)
            env[k.lstrip("-")] = v
    exe = _cached(TPF(), sanitize=False)
    for name in names:
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        rec = record(0, P.to_bytes(), blob, 7, 1 << 40, 64 * 64)
        r = subprocess.run([str(exe)], input=rec, capture_output=True, env=env)
        line = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("count record")]
        summ = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("records=")]
        ok = bool(summ) and " ok=1 " in summ[0]
        print(name, line[0].split(":", 1)[1].strip() if line else r.stdout.decode()[-300:] + r.stderr.decode()[-300:],
              "" if ok else "(DIFFERS from the C port: %s)" % (r.stdout.decode()[-400:]))
        # MYTHGPU_JIT_ASM_ANNOTATE=1: the program instructions costing the most VALU per candidate
        tags = []
        for ln in r.stdout.decode().splitlines():
            if ln.startswith("count tag "):
                t, v = ln[len("count tag "):].rsplit(":", 1)
                va, _, sa = v.strip().partition(" salu ")
                tags.append((float(va), float(sa or 0), t.strip()))
        key = (lambda x: x[1]) if env.get("ASMSIM_SORT") == "salu" else (lambda x: x[0])
        for v, sv, t in sorted(tags, key=key, reverse=True)[:int(env.get("ASMSIM_TOP", "40"))]:
            print(f"  {v:8.2f} {sv:8.2f}  {t}")


if __name__ == "__main__":
    main()
