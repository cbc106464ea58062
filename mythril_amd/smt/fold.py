"""Literal folding for the term mirror (the role ``z3.simplify`` plays for LASER's
``BitVec.value`` / ``Bool.__bool__`` checks, ``mythril/laser/smt/expression.py:37-39``).

Only nodes whose operands are all literals are folded; nothing symbolic is
rewritten.  This is host-side term construction, not constraint evaluation: the
engine never calls it on the get_model path (that path is GPU-only).
"""
from __future__ import annotations

from . import terms as T


def _s(v: int, w: int) -> int:
    return v - (1 << w) if v >> (w - 1) else v


def _udiv(a, b, w):
    return ((1 << w) - 1) if b == 0 else a // b


def _urem(a, b, w):
    return a if b == 0 else a % b


def _sdiv(a, b, w):
    sa, sb = _s(a, w), _s(b, w)
    if sb == 0:
        return 1 if sa < 0 else (1 << w) - 1
    q = abs(sa) // abs(sb)
    return (-q if (sa < 0) != (sb < 0) else q) % (1 << w)


def _srem(a, b, w):
    sa, sb = _s(a, w), _s(b, w)
    if sb == 0:
        return a
    r = abs(sa) % abs(sb)
    return (-r if sa < 0 else r) % (1 << w)


def _smod(a, b, w):
    sa, sb = _s(a, w), _s(b, w)
    if sb == 0:
        return a
    return (sa - sb * (sa // sb)) % (1 << w)  # Python floor-mod == SMT-LIB bvsmod


_BIN = {
    "bvadd": lambda a, b, w: (a + b),
    "bvsub": lambda a, b, w: (a - b),
    "bvmul": lambda a, b, w: (a * b),
    "bvudiv": _udiv,
    "bvurem": _urem,
    "bvsdiv": _sdiv,
    "bvsrem": _srem,
    "bvsmod": _smod,
    "bvand": lambda a, b, w: a & b,
    "bvor": lambda a, b, w: a | b,
    "bvxor": lambda a, b, w: a ^ b,
    "bvshl": lambda a, b, w: 0 if b >= w else a << b,
    "bvlshr": lambda a, b, w: 0 if b >= w else a >> b,
    "bvashr": lambda a, b, w: (_s(a, w) >> min(b, w)),
    "bvexp": lambda a, b, w: pow(a, b, 1 << w),
}

_CMP = {
    "bvult": lambda a, b, w: a < b,
    "bvule": lambda a, b, w: a <= b,
    "bvugt": lambda a, b, w: a > b,
    "bvuge": lambda a, b, w: a >= b,
    "bvslt": lambda a, b, w: _s(a, w) < _s(b, w),
    "bvsle": lambda a, b, w: _s(a, w) <= _s(b, w),
    "bvsgt": lambda a, b, w: _s(a, w) > _s(b, w),
    "bvsge": lambda a, b, w: _s(a, w) >= _s(b, w),
    "bvumul_noovfl": lambda a, b, w: a * b < (1 << w),
}


def fold(t: T.Term, _memo=None) -> T.Term:
    memo = {} if _memo is None else _memo
    return _fold(t, memo)


def _fold(t: T.Term, memo) -> T.Term:
    r = memo.get(t.id)
    if r is not None:
        return r
    if not t.args:
        memo[t.id] = t
        return t
    args = tuple(_fold(a, memo) for a in t.args)
    vals = [T.const_value(a) for a in args]
    res = None
    if all(v is not None for v in vals) and not any(a.is_array for a in args):
        op = t.op
        if op in _BIN:
            w = t.width
            res = T.BitVecVal(_BIN[op](vals[0], vals[1], w) % (1 << w), w)
        elif op in _CMP:
            res = T.BoolVal(_CMP[op](vals[0], vals[1], args[0].width))
        elif op == "bvnot":
            res = T.BitVecVal(~vals[0], t.width)
        elif op == "bvneg":
            res = T.BitVecVal(-vals[0], t.width)
        elif op == "concat":
            res = T.BitVecVal((vals[0] << args[1].width) | vals[1], t.width)
        elif op == "extract":
            hi, lo = t.params
            res = T.BitVecVal(vals[0] >> lo, hi - lo + 1)
        elif op == "zero_extend":
            res = T.BitVecVal(vals[0], t.width)
        elif op == "sign_extend":
            res = T.BitVecVal(_s(vals[0], args[0].width), t.width)
        elif op == "eq":
            res = T.BoolVal(vals[0] == vals[1])
        elif op == "not":
            res = T.BoolVal(not vals[0])
        elif op == "and":
            res = T.BoolVal(all(vals))
        elif op == "or":
            res = T.BoolVal(any(vals))
        elif op == "xor":
            res = T.BoolVal(bool(vals[0]) != bool(vals[1]))
        elif op == "ite":
            res = args[1] if vals[0] else args[2]
    elif t.op == "ite" and T.const_value(args[0]) is not None:
        res = args[1] if T.const_value(args[0]) else args[2]
    elif t.op == "select" and T.const_value(args[1]) is not None:
        # z3 simplify's array rewrite: Select(Store(a, i, v), j) with literal i, j is v
        # when i == j and Select(a, j) when i != j; K(v) reads v.  It stops at the first
        # symbolic store index (account.py:61 returns simplify(storage[item])).
        j = T.const_value(args[1])
        arr = args[0]
        while arr.op == "store" and T.const_value(arr.args[1]) is not None and T.const_value(arr.args[1]) != j:
            arr = arr.args[0]
        if arr.op == "store" and T.const_value(arr.args[1]) == j:
            res = arr.args[2]
        elif arr.op == "const_array":
            res = arr.args[0]
        elif arr is not args[0]:
            res = T.mk("select", t.sort, (arr, args[1]))
    elif t.op == "eq" and args[0] is args[1]:
        res = T.BoolVal(True)  # hash-consed: structurally equal (z3 simplify does the same)
    if res is None:
        res = t if args == t.args else T.mk(t.op, t.sort, args, t.params)
    memo[t.id] = res
    return res
