"""GPU microbenchmark of the generic interpreter (k_run): ns per interpreted op, per op
kind, from synthetic programs of N copies of one operation (chained, so nothing is dead
after specialisation).  Run on the GPU box:  python tools/interp_micro.py"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from mythril_amd import native, search, ssa  # noqa: E402
from mythril_amd.smt import terms as T  # noqa: E402


def chain(kind, n):
    x = T.BitVecVar("x", 256)
    y = T.BitVecVar("y", 256)
    b = T.BitVecVar("b", 8)
    acc = x
    roots = []
    for i in range(n):
        if kind == "add256":
            acc = T.bvbin("bvadd", acc, y)
        elif kind == "xor256":
            acc = T.bvbin("bvxor", acc, y)
        elif kind == "ult256":
            roots.append(T.not_(T.bvcmp("bvult", T.bvbin("bvadd", acc, T.BitVecVal(i, 256)), y)))
            acc = T.bvbin("bvadd", acc, T.BitVecVal(1, 256))
        elif kind == "eq256":
            roots.append(T.not_(T.eq(acc, T.BitVecVal(i + 12345, 256))))
            acc = T.bvbin("bvxor", acc, y)
        elif kind == "ite256":
            acc = T.ite(T.bvcmp("bvult", b, T.BitVecVal(i % 200, 8)), acc, T.bvbin("bvxor", acc, y))
        elif kind == "add8":
            b = T.bvbin("bvadd", b, T.BitVecVal(3, 8))
        elif kind == "mul256":
            acc = T.bvbin("bvmul", acc, y)
        elif kind == "extract":
            acc = T.zero_extend(248, T.extract(7 + (i % 8), i % 8, T.bvbin("bvadd", acc, y)))
        elif kind == "coord256":
            acc = T.bvbin("bvxor", acc, T.BitVecVar(f"c{i}", 256))
    if kind == "add8":
        roots.append(T.not_(T.eq(b, T.BitVecVal(7, 8))))
    roots.append(T.not_(T.eq(acc, T.BitVecVal(7, 256))))
    return roots


def main():
    eng = native.Engine.get()
    out = []
    for kind in ["add256", "xor256", "ult256", "eq256", "ite256", "add8", "mul256", "extract", "coord256"]:
        row = {"kind": kind}
        for n in (16, 96):
            roots = chain(kind, n)
            P, blob = search.prepare(roots)
            prog = eng.load(P.to_bytes())
            gh = eng.load_gen(prog, blob)
            info = eng.gen_info(gh)
            C = 1 << 22
            eng.search(prog, gh, 1, 0, C, early_exit=False)
            t = time.perf_counter()
            eng.search(prog, gh, 1, 0, C, early_exit=False)
            ms = eng.stats().last_kernel_ms
            row[f"n{n}"] = {"instrs": info.n_instrs, "words": info.value_words, "ms": ms}
            eng.free_gen(gh)
            eng.free(prog)
        a, b = row["n16"], row["n96"]
        d_instr = b["instrs"] - a["instrs"]
        # ns per interpreted instruction per 64-candidate wave at full chip
        row["ns_per_op_per_Mcand"] = (b["ms"] - a["ms"]) * 1e6 / max(d_instr, 1) / (C / 1e6)
        row["cand_per_s_at_n96"] = C / (b["ms"] * 1e-3)
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
