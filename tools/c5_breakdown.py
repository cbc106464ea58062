"""Where C5's (sha3_keyed_mapping) JIT time goes: kernel time per 2^24 candidates of the full
query and of its parts over the same coordinates (the kernel is VALU-bound, so time is
proportional to instructions).  GPU box: python tools/c5_breakdown.py"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from mythril_amd import native, search, workloads  # noqa: E402
from mythril_amd.smt import BitVec, Concat, ULT, symbol_factory  # noqa: E402
from mythril_amd.smt import terms as T  # noqa: E402

BVS, BVV = symbol_factory.BitVecSym, symbol_factory.BitVecVal
eng = native.Engine.get()


def kernel_ms(roots, n=1 << 24, reps=5):
    P, blob = search.prepare(roots)
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    jh = eng.jit_compile(prog, gh)
    try:
        eng.jit_search(jh, 1, 0, n, early_exit=False)
        eng.reset_stats()
        for r in range(reps):
            eng.jit_search(jh, 1, (r + 1) * n, n, early_exit=False)
        st = eng.stats()
        return st.kernel_ms_total / st.launches
    finally:
        eng.jit_free(jh)
        eng.free_gen(gh)
        eng.free(prog)


a = BVS("a", 256) & BVV((1 << 160) - 1, 256)
b, c, x, y = BVS("b", 256), BVS("c", 256), BVS("x", 256), BVS("y", 256)
d = BVS("d", 256) & BVV(0xFF, 256)
h1 = BitVec(T.keccak256(Concat(a, BVV(3, 256)).raw))
h2 = BitVec(T.keccak256(Concat(h1, b).raw))
e = BitVec(T.bvexp(c.raw, d.raw))
parts = {
    "full": [c_.raw for c_ in workloads.WORKLOADS["sha3_keyed_mapping"]()],
    "keccak2": [ULT(h2, BVV(1 << 240, 256)).raw],
    "keccak1": [ULT(h1, BVV(1 << 240, 256)).raw],
    "exp_sdiv": [((x / y) < (e / BVV(3, 256))).raw],
    "exp": [ULT(e, BVV(1 << 200, 256)).raw],
    "sdiv_xy": [((x / y) < BVV(5, 256)).raw],
    "gen_only": [ULT(x ^ y ^ b ^ c ^ d ^ a, BVV(1 << 255, 256)).raw],
}
out = {k: round(kernel_ms(v), 4) for k, v in parts.items()}
print(json.dumps(out))
