"""ORACLE (test infrastructure only) — z3 ``model.eval(expr, model_completion=True)``
restated over Python integers.

What it restates.  The reference hands every path constraint to z3 and reads
values back with ``Model.eval`` (``mythril/laser/smt/model.py:45-59``,
``mythril/support/model.py:15-49``).  z3 (``z3-solver>=4.8.5.0``,
``requirements.txt:30``, not vendored and not installed here) implements the
SMT-LIB ``QF_ABV`` theory; this module restates that published semantics for the
exact vocabulary LASER emits:

* total division (SMT-LIB FixedSizeBitVectors): ``bvudiv x 0 = ~0``,
  ``bvurem x 0 = x``; ``bvsdiv``/``bvsrem``/``bvsmod`` defined through the msb
  case split of the standard; shifts by >= w give 0 (``bvshl``/``bvlshr``) or
  sign fill (``bvashr``);
* ``bvumul_noovfl``: the 2w-bit product fits in w bits (z3 primitive used by
  ``BVMulNoOverflow``, ``bitvec_helper.py:183-196``);
* arrays and uninterpreted functions under a finite model: an explicit
  ``{index: value}`` table plus an ``else`` value (z3 ``as-array``/``FuncInterp``);
  with model completion, an unassigned symbol evaluates to 0;
* EVM extensions used by replay programs: ``keccak256`` (``oracle/keccak.py``)
  and ``bvexp`` (``pow(b, e, 2**w)``, ``mythril/laser/ethereum/instructions.py:599-631``).

Parity status: the z3 boundary itself cannot be run in this image (no z3, no
network), so evaluation exactness is pinned through the reference's golden
vectors (VMTests post-states, EIP-145 shift vectors, Keccak KATs — see
``tests/golden/``) rather than against z3 directly.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline may
import this module.
"""
from __future__ import annotations

from typing import Dict, Iterable

from oracle.keccak import keccak256_int


class OracleModel:
    """A finite z3-style model: scalars, array tables and function tables."""

    def __init__(self, scalars=None, arrays=None, funcs=None):
        self.scalars: Dict[str, int] = dict(scalars or {})
        # name -> (table, else_value)
        self.arrays: Dict[str, tuple] = dict(arrays or {})
        self.funcs: Dict[str, tuple] = dict(funcs or {})


def _mask(w):
    return (1 << w) - 1


def _msb(v, w):
    return (v >> (w - 1)) & 1


def _neg(v, w):
    return (-v) & _mask(w)


def bvudiv(s, t, w):
    if t == 0:
        return _mask(w)
    return s // t


def bvurem(s, t, w):
    if t == 0:
        return s
    return s % t


def bvsdiv(s, t, w):
    # SMT-LIB:  (ite (and (= msb_s #b0) (= msb_t #b0)) (bvudiv s t)
    #           (ite (and (= msb_s #b1) (= msb_t #b0)) (bvneg (bvudiv (bvneg s) t))
    #           (ite (and (= msb_s #b0) (= msb_t #b1)) (bvneg (bvudiv s (bvneg t)))
    #                (bvudiv (bvneg s) (bvneg t)))))
    ms, mt = _msb(s, w), _msb(t, w)
    if not ms and not mt:
        return bvudiv(s, t, w)
    if ms and not mt:
        return _neg(bvudiv(_neg(s, w), t, w), w)
    if not ms and mt:
        return _neg(bvudiv(s, _neg(t, w), w), w)
    return bvudiv(_neg(s, w), _neg(t, w), w)


def bvsrem(s, t, w):
    ms, mt = _msb(s, w), _msb(t, w)
    if not ms and not mt:
        return bvurem(s, t, w)
    if ms and not mt:
        return _neg(bvurem(_neg(s, w), t, w), w)
    if not ms and mt:
        return bvurem(s, _neg(t, w), w)
    return _neg(bvurem(_neg(s, w), _neg(t, w), w), w)


def bvsmod(s, t, w):
    ms, mt = _msb(s, w), _msb(t, w)
    abs_s = _neg(s, w) if ms else s
    abs_t = _neg(t, w) if mt else t
    u = bvurem(abs_s, abs_t, w)
    if u == 0:
        return u
    if not ms and not mt:
        return u
    if ms and not mt:
        return (_neg(u, w) + t) & _mask(w)
    if not ms and mt:
        return (u + t) & _mask(w)
    return _neg(u, w)


def _signed(v, w):
    return v - (1 << w) if _msb(v, w) else v


def bvshl(a, b, w):
    return 0 if b >= w else (a << b) & _mask(w)


def bvlshr(a, b, w):
    return 0 if b >= w else a >> b


def bvashr(a, b, w):
    if b >= w:
        return _mask(w) if _msb(a, w) else 0
    return (_signed(a, w) >> b) & _mask(w)


_BIN = {
    "bvadd": lambda a, b, w: (a + b) & _mask(w),
    "bvsub": lambda a, b, w: (a - b) & _mask(w),
    "bvmul": lambda a, b, w: (a * b) & _mask(w),
    "bvudiv": bvudiv,
    "bvurem": bvurem,
    "bvsdiv": bvsdiv,
    "bvsrem": bvsrem,
    "bvsmod": bvsmod,
    "bvand": lambda a, b, w: a & b,
    "bvor": lambda a, b, w: a | b,
    "bvxor": lambda a, b, w: a ^ b,
    "bvshl": bvshl,
    "bvlshr": bvlshr,
    "bvashr": bvashr,
    "bvexp": lambda a, b, w: pow(a, b, 1 << w),
}

_CMP = {
    "bvult": lambda a, b, w: a < b,
    "bvule": lambda a, b, w: a <= b,
    "bvugt": lambda a, b, w: a > b,
    "bvuge": lambda a, b, w: a >= b,
    "bvslt": lambda a, b, w: _signed(a, w) < _signed(b, w),
    "bvsle": lambda a, b, w: _signed(a, w) <= _signed(b, w),
    "bvsgt": lambda a, b, w: _signed(a, w) > _signed(b, w),
    "bvsge": lambda a, b, w: _signed(a, w) >= _signed(b, w),
    "bvumul_noovfl": lambda a, b, w: a * b <= _mask(w),
}


class _ArrayVal:
    """Value of an array term under a model: a chain of stores over a base."""

    __slots__ = ("stores", "base_name", "base_default")

    def __init__(self, stores, base_name, base_default):
        self.stores = stores          # list of (idx, val), newest last
        self.base_name = base_name    # array variable name or None
        self.base_default = base_default

    def read(self, model: OracleModel, idx: int) -> int:
        for i, v in reversed(self.stores):
            if i == idx:
                return v
        if self.base_name is None:
            return self.base_default
        table, dflt = model.arrays.get(self.base_name, ({}, 0))
        return table.get(idx, dflt)


def evaluate(term, model: OracleModel, memo=None) -> int:
    """Evaluate one term; Bools come back as 0/1."""
    return evaluate_many([term], model, memo)[0]


def evaluate_many(roots: Iterable, model: OracleModel, memo=None):
    from mythril_amd.smt.terms import postorder  # the term format under test

    memo = {} if memo is None else memo
    roots = list(roots)
    for t in postorder(roots):
        if t.id in memo:
            continue
        memo[t.id] = _eval_node(t, model, memo)
    return [memo[r.id] for r in roots]


def _eval_node(t, model: OracleModel, memo):
    op = t.op
    a = [memo[x.id] for x in t.args]
    if op == "bvconst":
        return t.params[0]
    if op == "boolconst":
        return int(t.params[0])
    if op in ("bvvar", "boolvar"):
        return model.scalars.get(t.params[0], 0) & _mask(t.width)
    if op in _BIN:
        return _BIN[op](a[0], a[1], t.width)
    if op in _CMP:
        return int(_CMP[op](a[0], a[1], t.args[0].width))
    if op == "bvnot":
        return ~a[0] & _mask(t.width)
    if op == "bvneg":
        return _neg(a[0], t.width)
    if op == "concat":
        return (a[0] << t.args[1].width) | a[1]
    if op == "extract":
        hi, lo = t.params
        return (a[0] >> lo) & _mask(hi - lo + 1)
    if op == "zero_extend":
        return a[0]
    if op == "sign_extend":
        w0 = t.args[0].width
        return _signed(a[0], w0) & _mask(t.width)
    if op == "ite":
        return a[1] if a[0] else a[2]
    if op == "eq":
        return int(a[0] == a[1])
    if op == "not":
        return int(not a[0])
    if op == "and":
        return int(all(a))
    if op == "or":
        return int(any(a))
    if op == "xor":
        return int(bool(a[0]) != bool(a[1]))
    if op == "array_var":
        return _ArrayVal([], t.params[0], 0)
    if op == "const_array":
        return _ArrayVal([], None, a[0])
    if op == "store":
        base = a[0]
        return _ArrayVal(base.stores + [(a[1], a[2])], base.base_name, base.base_default)
    if op == "select":
        return a[0].read(model, a[1])
    if op == "app":
        table, dflt = model.funcs.get(t.params[0], ({}, 0))
        return table.get(a[0], dflt) & _mask(t.width)
    if op == "keccak256":
        if not t.args:
            return keccak256_int(b"")
        w = t.args[0].width
        return keccak256_int(a[0].to_bytes(w // 8, "big"))
    raise NotImplementedError(f"oracle: operator {op}")


def model_from_coordinates(P, assignment):
    """The finite model a candidate denotes: scalars from their coordinates; each
    array/UF site, in SSA order, adds ``key -> coordinate`` (or its lazy default)
    unless an earlier site of the same table already holds that key.  This is the
    z3-model reading of a candidate that the engine's canonicalisation implements
    (mythril_amd/ssa.py docstring); restated here independently for the tests."""
    def mask(v, w):
        return v & ((1 << w) - 1)

    scal = {c.name: mask(assignment[c.index], c.width) for c in P.scalar_coords()}
    arrays, funcs = {}, {}
    for c in P.sites:
        m = OracleModel(scal, arrays, funcs)
        key = evaluate(P.node_term[P.site_key_node[c.index]], m)
        lazy = P.nodes[c.node][7] if c.kind == 2 else 0xFFFFFFFF
        if lazy != 0xFFFFFFFF:
            dflt = evaluate(P.node_term[lazy], m)
        else:
            dflt = mask(assignment[c.index], c.width)
        tables = arrays if c.kind == 1 else funcs
        table, _ = tables.setdefault(c.name, ({}, 0))
        table.setdefault(key, dflt)
    return OracleModel(scal, arrays, funcs)
