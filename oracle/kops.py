"""ORACLE (test infrastructure only) — a plain-Python evaluator of the engine's *lowered,
specialised* program (``mg_program_specialized``: the device ops of
``mythril_amd/csrc/program.hpp`` over SSA value ids).

It exists to check one claim of the engine on CPU: specialisation (range-decided compares,
aliases, dead code; ``program.cpp: specialize_program``) keeps the verdict of every
candidate the generator can draw.  ``tests/test_specialize_cpu.py`` runs the specialised
program here on the candidates ``oracle/bveval.c`` generates (``bv_gen_soa``) and compares
with the C port's verdicts on the *unspecialised* program.  The op semantics restate
z3's ``model.eval`` for the QF_ABV vocabulary (SMT-LIB total division, saturating shifts),
as ``oracle/bv.py`` does for terms.  Never imported by the product.
"""
from typing import Dict, List, Sequence

import numpy as np

from oracle.keccak import keccak256

NONE = 0xFFFFFFFF
(K_CONST, K_COORD, K_ADD, K_SUB, K_MUL, K_UDIV, K_UREM, K_SDIV, K_SREM, K_SMOD, K_AND, K_OR, K_XOR, K_NOT, K_NEG,
 K_SHL, K_LSHR, K_ASHR, K_CONCAT, K_EXTRACT, K_ZEXT, K_SEXT, K_ITE, K_EQ, K_ULT, K_ULE, K_SLT, K_SLE,
 K_UMUL_NOOVF, K_EXP, K_LOOKUP, K_KECCAK, K_ASSERT, K_WATCH, K_COPY) = range(35)


def _limbs_to_int(words: Sequence[int]) -> int:
    v = 0
    for j, x in enumerate(words):
        v |= int(x) << (32 * j)
    return v


def _signed(x: int, w: int) -> int:
    return x - (1 << w) if x >> (w - 1) & 1 else x


def _udiv(a: int, b: int, m: int) -> int:
    return m if b == 0 else a // b


def _urem(a: int, b: int) -> int:
    return a if b == 0 else a % b


def _sdivrem(op: int, a: int, b: int, w: int) -> int:
    m = (1 << w) - 1
    sa, sb = a >> (w - 1) & 1, b >> (w - 1) & 1
    aa = (-a) & m if sa else a
    bb = (-b) & m if sb else b
    q, r = (m, aa) if bb == 0 else divmod(aa, bb)
    if op == K_SDIV:
        return (-q) & m if sa ^ sb else q
    if op == K_SREM:
        return (-r) & m if sa else r
    # SMOD: sign of the divisor
    if r == 0 or (not sa and not sb):
        return r
    if sa and not sb:
        return ((-r) + b) & m
    if not sa and sb:
        return (r + b) & m
    return (-r) & m


def run(spec: Dict, coords: List[int]) -> int:
    """Verdict (0/1) of one candidate; ``coords[c]`` = the value of coordinate c."""
    code, consts, aux, widths = spec["code"], spec["consts"], spec["aux"], spec["widths"]
    val: Dict[int, int] = {}
    verdict = 1
    for row in code:
        op, W, d, a, b, c, p0, p1 = (int(x) for x in row)
        m = (1 << W) - 1 if W else 0
        A = val.get(a) if a != NONE else None
        B = val.get(b) if b != NONE else None
        if op == K_CONST:
            r = _limbs_to_int(consts[p0:p0 + (W + 31) // 32]) & m
        elif op == K_COORD:
            r = coords[p0] & m
        elif op == K_COPY:
            r = A
        elif op == K_ADD:
            r = (A + B) & m
        elif op == K_SUB:
            r = (A - B) & m
        elif op == K_NEG:
            r = (-A) & m
        elif op == K_MUL:
            r = (A * B) & m
        elif op == K_UDIV:
            r = _udiv(A, B, m)
        elif op == K_UREM:
            r = _urem(A, B)
        elif op in (K_SDIV, K_SREM, K_SMOD):
            r = _sdivrem(op, A, B, W)
        elif op == K_AND:
            r = A & B
        elif op == K_OR:
            r = A | B
        elif op == K_XOR:
            r = A ^ B
        elif op == K_NOT:
            r = ~A & m
        elif op == K_SHL:
            r = 0 if B >= W else (A << B) & m
        elif op == K_LSHR:
            r = 0 if B >= W else A >> B
        elif op == K_ASHR:
            r = (_signed(A, W) >> min(B, W)) & m
        elif op == K_CONCAT:
            r = (A << p1) | B
        elif op == K_EXTRACT:
            r = (A >> p0) & m
        elif op == K_ZEXT:
            r = A
        elif op == K_SEXT:
            r = _signed(A, p1) & m
        elif op == K_ITE:
            r = B if A else val[c]
        elif op == K_EQ:
            r = int(A == B)
        elif op == K_ULT:
            r = int(A < B)
        elif op == K_ULE:
            r = int(A <= B)
        elif op == K_SLT:
            r = int(_signed(A, p1) < _signed(B, p1))
        elif op == K_SLE:
            r = int(_signed(A, p1) <= _signed(B, p1))
        elif op == K_UMUL_NOOVF:
            r = int(A * B < (1 << p1))
        elif op == K_EXP:
            r = pow(A, B, 1 << W)
        elif op == K_LOOKUP:
            r = val[p0]
            for k in range(c):  # first prior whose key equals a
                kv, vv = int(aux[p1 + 2 * k]), int(aux[p1 + 2 * k + 1])
                if val[kv] == A:
                    r = val[vv]
                    break
        elif op == K_KECCAK:
            data = b"" if a == NONE else A.to_bytes(p0, "big")
            r = int.from_bytes(keccak256(data), "big")
        elif op == K_ASSERT:
            verdict &= A & 1
            continue
        elif op == K_WATCH:
            continue
        else:
            raise ValueError(f"unknown device op {op}")
        val[d] = r
    return verdict


def coords_from_soa(soa: np.ndarray, widths: Sequence[int], i: int) -> List[int]:
    """Coordinate values of SoA column i (rows of ceil(w/32) limbs per coordinate, in order)."""
    out, row = [], 0
    for w in widths:
        L = (w + 31) // 32
        out.append(_limbs_to_int(soa[row:row + L, i]))
        row += L
    return out


def verdicts(spec: Dict, soa: np.ndarray, coord_widths: Sequence[int], n: int) -> np.ndarray:
    return np.array([run(spec, coords_from_soa(soa, coord_widths, i)) for i in range(n)], dtype=np.uint8)
