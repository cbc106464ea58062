"""Phase split of the JIT's cold compile on this host (no GPU needed; run on the box's host
for the numbers that matter).  For each workload's search kernel:

* comgr, as the engine calls it (in-process, its cache off): source -> bitcode (clang front end
  + the LLVM optimiser), bitcode -> relocatable (machine code generation), link;
* the same source through the standalone clang with ``-ftime-report``: front end, IR
  generation, optimiser, machine code generation;
* the asm tier (``mg_program_jit_asm``, jit_asm.cpp): emission, and assembly + link through
  comgr, when the program is inside that tier.

  python tools/jit_phases.py [workload ...] > profiles/rNN_jit_phases.jsonl
"""
import json
import os
import re
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

CHILD = r"""
import sys, time
sys.path.insert(0, %r)
from mythril_amd import native, search, workloads
name = sys.argv[1]
roots = [c.raw for c in workloads.WORKLOADS[name]()]
P, blob = search.prepare(roots)
t = time.perf_counter(); src = native.jit_source(P.to_bytes(), blob); t_emit = time.perf_counter() - t
open(sys.argv[2], "w").write(src)
t = time.perf_counter(); native.jit_source(P.to_bytes(), blob, compile=True); t_all = time.perf_counter() - t
print("EMIT %%.3f ALL %%.3f" %% (t_emit * 1e3, t_all * 1e3))
try:
    t = time.perf_counter(); asm = native.jit_asm(P.to_bytes(), blob); t_asm = time.perf_counter() - t
    t = time.perf_counter(); native.jit_asm(P.to_bytes(), blob, compile=True); t_asm_all = time.perf_counter() - t
    print("ASM %%.3f ASMALL %%.3f LINES %%d" %% (t_asm * 1e3, t_asm_all * 1e3, asm.count(chr(10))))
except Exception as e:
    print("ASMERR", str(e)[:200].replace(chr(10), " "))
""" % str(ROOT)


def shim_source() -> str:
    s = (ROOT / "mythril_amd/csrc/jit.cpp").read_text()
    a = s.index('const char* kComgrShim = R"MGJ(') + len('const char* kComgrShim = R"MGJ(')
    return s[a:s.index(')MGJ"', a)]


def clang_split(src_path: str) -> dict:
    full = tempfile.NamedTemporaryFile("w", suffix=".hip", delete=False)
    full.write(shim_source() + open(src_path).read())
    full.close()
    cmd = ["/opt/rocm/lib/llvm/bin/clang", "-x", "hip", "--cuda-device-only", "--offload-arch=gfx950", "-O3",
           "-std=c++17", "-nogpuinc", "-nogpulib", "-fno-slp-vectorize", "-fno-unroll-loops", "-mllvm",
           "-structurizecfg-skip-uniform-regions", "-Wno-unused-variable", "-Wno-uninitialized",
           "-Wno-sometimes-uninitialized", "-c", full.name, "-o", os.devnull, "-ftime-report"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    os.unlink(full.name)
    out = {}
    i = r.stderr.find("Clang time report")
    for line in r.stderr[i:].splitlines()[4:12] if i >= 0 else []:
        m = re.match(r"\s*[\d.]+ \(.*?\)\s+[\d.]+ \(.*?\)\s+[\d.]+ \(.*?\)\s+([\d.]+) \(.*?\)\s+(.*)$", line)
        if m and m.group(2).strip() != "Total":
            out[m.group(2).strip()] = round(float(m.group(1)) * 1e3, 2)
    return out


def main():
    from mythril_amd import workloads

    names = sys.argv[1:] or sorted(workloads.WORKLOADS)
    host = {"nproc": os.cpu_count()}
    try:
        host["cpu"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        pass
    env = dict(os.environ, MYTHGPU_JIT_TIMING="1", MYTHGPU_JIT_ISOLATE="0", AMD_COMGR_CACHE="0",
               MYTHGPU_JIT_DISK_CACHE="0")
    for name in names:
        with tempfile.NamedTemporaryFile(suffix=".hip", delete=False) as f:
            src_path = f.name
        t = time.perf_counter()
        r = subprocess.run([sys.executable, "-c", CHILD, name, src_path], capture_output=True, text=True, env=env)
        rec = {"workload": name, "host": host, "source_bytes": os.path.getsize(src_path)}
        m = re.search(r"front\+opt ([\d.]+) ms, codegen ([\d.]+) ms, link ([\d.]+) ms", r.stderr)
        if m:
            rec["comgr_ms"] = {"source_to_bc": float(m.group(1)), "bc_to_relocatable": float(m.group(2)),
                               "link": float(m.group(3))}
        m = re.search(r"EMIT ([\d.]+) ALL ([\d.]+)", r.stdout)
        if m:
            rec["emit_ms"], rec["compile_total_ms"] = float(m.group(1)), float(m.group(2))
        m = re.search(r"ASM ([\d.]+) ASMALL ([\d.]+) LINES (\d+)", r.stdout)
        if m:
            rec["asm_tier"] = {"emit_ms": float(m.group(1)), "emit_assemble_link_ms": float(m.group(2)),
                               "lines": int(m.group(3))}
        m = re.search(r"ASMERR (.*)", r.stdout)
        if m:
            rec["asm_tier"] = {"unsupported": m.group(1)}
        if r.returncode != 0:
            rec["error"] = r.stderr[-500:]
        rec["clang_time_report_ms"] = clang_split(src_path)
        os.unlink(src_path)
        rec["wall_s"] = round(time.perf_counter() - t, 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
