"""Host-only: per-basic-block instruction counts of a JIT kernel (after tools/jit_disasm.py
wrote /tmp/jd/<workload>.co).  Shows where the static VALU instructions of mgj_search sit:
the generator's alternatives are the blocks between SGPR branches, the straight-line
evaluation is the long blocks.
usage: python tools/jit_blocks.py [workload] [kernel]"""
import re
import subprocess
import sys

name = sys.argv[1] if len(sys.argv) > 1 else "token_transfer_underflow"
kern = sys.argv[2] if len(sys.argv) > 2 else "mgj_search"
dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--symbolize-operands", f"/tmp/jd/{name}.co"],
                     capture_output=True, text=True).stdout.split("\n")
start = next(i for i, l in enumerate(dis) if re.match(rf"^[0-9a-f]+ <{kern}>:", l))
blocks = [["entry", 0, 0, 0, 0, []]]
for l in dis[start + 1:]:
    if re.match(r"^[0-9a-f]+ <mgj_", l):
        break
    m = re.match(r"^[0-9a-f]+ <(L\d+)>:", l)
    if m:
        blocks.append([m.group(1), 0, 0, 0, 0, []])
        continue
    m = re.match(r"^\s+([a-z][a-z0-9_]+)\s*([^/]*)", l)
    if not m:
        continue
    op, args, cur = m.group(1), m.group(2).strip(), blocks[-1]
    if op.startswith("v_"):
        cur[1] += 1
    elif op == "s_nop":
        cur[4] += 1
    elif op.startswith("s_cbranch") or op == "s_branch":
        cur[5].append(f"{op[2:]} {args}")
    elif op.startswith("s_"):
        cur[2] += 1
    else:
        cur[3] += 1
tot = [0, 0, 0, 0]
for b in blocks:
    print(f"{b[0]:>6} VALU {b[1]:4d} SALU {b[2]:4d} MEM {b[3]:3d} NOP {b[4]:3d}  -> {'; '.join(b[5])}")
    for k in range(4):
        tot[k] += b[k + 1]
print("total VALU/SALU/MEM/NOP", tot)
