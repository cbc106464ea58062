"""Instructions per candidate of the O3 tier's search kernel on the CPU simulator (tests/asmsim):
the kernel is compiled as the engine compiles it (comgr, no GPU), disassembled by tools/o3dis.py and
run over a window of 64-candidate groups with full evaluation, its hits checked against the C port.
VALU / SALU lane-instructions per candidate (SQ_INSTS_VALU x 64 / candidates) and LDS bank-conflict
cycles (SQ_LDS_BANK_CONFLICT) per 64 candidates, without a GPU.

  python tools/o3_count.py [workload ...] [--lines] [--top N] [K=V ...]

--lines: compile with line tables and print the source statements costing the most VALU."""
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def o3_kernel(name, env, lines=False, tmp=None):
    """(sim text, O3 source, shim lines) of workload `name`'s search kernel"""
    tmp = tmp or tempfile.mkdtemp(prefix="o3count")
    pre = os.path.join(tmp, name)
    e = dict(env, MYTHGPU_JIT_DUMP=pre)
    if lines:
        e["MYTHGPU_JIT_EXTRA"] = (e.get("MYTHGPU_JIT_EXTRA", "") + " -gline-tables-only").strip()
    code = ("from mythril_amd import search, workloads, native\n"
            "P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[%r]()])\n"
            "native.jit_source(P.to_bytes(), blob, compile=True)\n" % name)
    subprocess.run([sys.executable, "-c", code], env=e, cwd=str(ROOT), check=True)
    from tools.o3dis import convert
    return convert(pre + ".co", lines=lines), Path(pre + ".hip").read_text()


def main():
    from mythril_amd import search, workloads
    from tests.test_asm_sim import _cached, record

    class TPF:
        def mktemp(self, name):
            return Path(tempfile.mkdtemp(prefix=name))

    args = sys.argv[1:]
    lines = "--lines" in args
    top = 30
    if "--top" in args:
        top = int(args[args.index("--top") + 1])
    env = dict(os.environ)
    names = []
    skip = False
    for i, a in enumerate(args):
        if skip:
            skip = False
            continue
        if a == "--top":
            skip = True
        elif a.startswith("--"):
            continue
        elif "=" in a:
            k, v = a.split("=", 1)
            env[k] = v
        else:
            names.append(a)
    names = names or sorted(workloads.WORKLOADS)
    exe = _cached(TPF(), sanitize=False)
    tmp = tempfile.mkdtemp(prefix="o3count")
    for name in names:
        text, src = o3_kernel(name, env, lines, tmp)
        sp = os.path.join(tmp, name + ".s")
        Path(sp).write_text(text)
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        rec = record(0, P.to_bytes(), blob, 7, 1 << 40, 64 * 64)
        r = subprocess.run([str(exe)], input=rec, capture_output=True,
                           env=dict(env, ASMSIM_COUNT="1", ASMSIM_SEARCH_SOURCE=sp))
        out = r.stdout.decode()
        cnt = [ln for ln in out.splitlines() if ln.startswith("count record")]
        summ = [ln for ln in out.splitlines() if ln.startswith("records=")]
        ok = bool(summ) and " ok=1 " in summ[0]
        print(name, cnt[0].split(":", 1)[1].strip() if cnt else out[-300:] + r.stderr.decode()[-300:],
              "" if ok else "(hits DIFFER from the C port: %s)" % (summ[0] if summ else "?"))
        if lines:
            srcl = src.splitlines()
            # the comgr shim's lines come first: the kernel's signature line locates the offset
            sig = next(i for i, l in enumerate(srcl, 1) if "mgj_search(" in l)
            first = int(re.search(r"; vcode line (\d+)", text).group(1))
            off = first - sig
            rows = []
            for ln in out.splitlines():
                if ln.startswith("count tag vcode line "):
                    a, v = ln[len("count tag vcode line "):].rsplit(":", 1)
                    v = v.split(" salu ")[0]
                    n = int(a) - off
                    rows.append((float(v), n, srcl[n - 1][:140] if 0 < n <= len(srcl) else "?"))
            for v, n, t in sorted(rows, reverse=True)[:top]:
                print("  %7.2f %5d %s" % (v, n, t))


if __name__ == "__main__":
    main()
