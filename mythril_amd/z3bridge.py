"""z3 AST -> engine terms (used inside a real Mythril process, where LASER's
``Bool``/``BitVec`` wrap z3 ASTs, ``mythril/laser/smt/expression.py:10-33``).

Hash-consed by ``get_id()``; iterative (LASER DAGs are deep).  Every z3
operator kind LASER's terms can reach after ``z3.simplify`` is mapped; anything
else raises :class:`Unsupported` and the query stays on z3.  This module needs
z3; the GPU box image has none, so it is exercised only where Mythril runs.
"""
from __future__ import annotations

from typing import Dict, List

from .smt import terms as T
from .ssa import Unsupported

try:
    import z3  # type: ignore
except Exception:  # pragma: no cover
    z3 = None


def _ops():
    k = {}
    names = {
        "BADD": "add", "BSUB": "sub", "BMUL": "mul", "BUDIV": "bvudiv", "BUDIV_I": "bvudiv",
        "BUREM": "bvurem", "BUREM_I": "bvurem", "BSDIV": "bvsdiv", "BSDIV_I": "bvsdiv",
        "BSREM": "bvsrem", "BSREM_I": "bvsrem", "BSMOD": "bvsmod", "BSMOD_I": "bvsmod",
        "BAND": "band", "BOR": "bor", "BXOR": "bxor", "BNOT": "bvnot", "BNEG": "bvneg",
        "BSHL": "bvshl", "BLSHR": "bvlshr", "BASHR": "bvashr", "CONCAT": "concat",
        "EXTRACT": "extract", "ZERO_EXT": "zero_extend", "SIGN_EXT": "sign_extend", "ITE": "ite",
        "EQ": "eq", "DISTINCT": "distinct", "ULEQ": "bvule", "UGEQ": "bvuge", "ULT": "bvult",
        "UGT": "bvugt", "SLEQ": "bvsle", "SGEQ": "bvsge", "SLT": "bvslt", "SGT": "bvsgt",
        "AND": "and", "OR": "or", "NOT": "not", "XOR": "xor", "IMPLIES": "implies", "IFF": "eq",
        "BUMUL_NO_OVFL": "bvumul_noovfl", "SELECT": "select", "STORE": "store",
        "CONST_ARRAY": "const_array", "TRUE": "true", "FALSE": "false", "BNUM": "bnum",
        "UNINTERPRETED": "uninterpreted",
    }
    for n, v in names.items():
        code = getattr(z3, "Z3_OP_" + n, None)
        if code is not None:
            k[code] = v
    return k


_OPS = None


def to_terms(exprs: List) -> List[T.Term]:
    """Convert z3 BoolRefs (or mythril ``Bool`` wrappers) to engine terms."""
    global _OPS
    if z3 is None:
        raise Unsupported("z3 is not importable")
    if _OPS is None:
        _OPS = _ops()
    memo: Dict[int, T.Term] = {}
    raws = [getattr(e, "raw", e) for e in exprs]
    stack = [(r, False) for r in raws]
    while stack:
        e, done = stack.pop()
        eid = e.get_id()
        if eid in memo:
            continue
        kids = [e.arg(i) for i in range(e.num_args())]
        if not done:
            stack.append((e, True))
            for c in kids:
                if c.get_id() not in memo:
                    stack.append((c, False))
            continue
        memo[eid] = _convert(e, [memo[c.get_id()] for c in kids])
    return [memo[r.get_id()] for r in raws]


def _sort_of(s):
    if s.kind() == z3.Z3_BOOL_SORT:
        return ("bool",)
    if s.kind() == z3.Z3_BV_SORT:
        return ("bv", s.size())
    if s.kind() == z3.Z3_ARRAY_SORT:
        d, r = s.domain(), s.range()
        if d.kind() != z3.Z3_BV_SORT or r.kind() != z3.Z3_BV_SORT:
            raise Unsupported("array sort")
        return ("array", d.size(), r.size())
    raise Unsupported(f"sort {s}")


def _fold(op, args):
    acc = args[0]
    for a in args[1:]:
        acc = T.bvbin(op, acc, a)
    return acc


def _convert(e, a: List[T.Term]) -> T.Term:
    decl = e.decl()
    kind = _OPS.get(decl.kind())
    if z3.is_bv_value(e):
        return T.BitVecVal(e.as_long(), e.size())
    if kind == "true":
        return T.BoolVal(True)
    if kind == "false":
        return T.BoolVal(False)
    if kind == "uninterpreted":
        name = decl.name()
        if e.num_args() == 0:
            srt = _sort_of(e.sort())
            if srt[0] == "bool":
                return T.BoolVar(name)
            if srt[0] == "bv":
                return T.BitVecVar(name, srt[1])
            return T.ArrayVar(name, srt[1], srt[2])
        if e.num_args() == 1:
            dom, rng = decl.domain(0), decl.range()
            if dom.kind() != z3.Z3_BV_SORT or rng.kind() != z3.Z3_BV_SORT:
                raise Unsupported("uninterpreted function sort")
            return T.app(T.FuncDecl(name, dom.size(), rng.size()), a[0])
        raise Unsupported("n-ary uninterpreted function")
    if kind in ("add", "mul", "band", "bor", "bxor"):
        return _fold({"add": "bvadd", "mul": "bvmul", "band": "bvand", "bor": "bvor", "bxor": "bvxor"}[kind], a)
    if kind == "sub":
        return _fold("bvsub", a)
    if kind in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvshl", "bvlshr", "bvashr"):
        return T.bvbin(kind, a[0], a[1])
    if kind in ("bvnot", "bvneg"):
        return T.bvun(kind, a[0])
    if kind in ("bvule", "bvuge", "bvult", "bvugt", "bvsle", "bvsge", "bvslt", "bvsgt", "bvumul_noovfl"):
        return T.bvcmp(kind, a[0], a[1])
    if kind == "concat":
        return T.concat(*a)
    if kind == "extract":
        hi, lo = decl.params()
        return T.extract(hi, lo, a[0])
    if kind == "zero_extend":
        return T.zero_extend(decl.params()[0], a[0])
    if kind == "sign_extend":
        return T.sign_extend(decl.params()[0], a[0])
    if kind == "ite":
        return T.ite(a[0], a[1], a[2])
    if kind == "eq":
        return T.eq(a[0], a[1])
    if kind == "distinct":
        return T.and_(*[T.not_(T.eq(a[i], a[j])) for i in range(len(a)) for j in range(i + 1, len(a))])
    if kind == "and":
        return T.and_(*a)
    if kind == "or":
        return T.or_(*a)
    if kind == "not":
        return T.not_(a[0])
    if kind == "xor":
        return T.xor_(a[0], a[1])
    if kind == "implies":
        return T.or_(T.not_(a[0]), a[1])
    if kind == "select":
        return T.select(a[0], a[1])
    if kind == "store":
        return T.store(a[0], a[1], a[2])
    if kind == "const_array":
        d = e.sort().domain().size()
        return T.ConstArray(d, a[0])
    raise Unsupported(f"z3 operator {decl.name()} (kind {decl.kind()})")


def pin_model(constraints, model, timeout_ms=None):
    """Re-check a GPU model with z3 and return a real ``z3.ModelRef``: the original
    constraints plus equalities pinning every symbol the GPU assigned (scalars,
    array table entries, function table entries).

    Runs in a fresh ``z3.Context`` (the constraints are translated into it), so LASER's
    main context and its solvers see no new assertions or declarations; the model is
    translated back to the main context for ``Model.eval``.  ``timeout_ms`` bounds the
    check (the caller passes what is left of the query's budget); ``unknown`` -> None,
    and the caller falls back to the original z3 path."""
    ctx = z3.Context()
    s = z3.Solver(ctx=ctx)
    if timeout_ms is not None:
        s.set("timeout", max(1, int(timeout_ms)))
    raws = [getattr(c, "raw", c).translate(ctx) for c in constraints]
    s.add(*raws)
    syms = {}
    for r in raws:
        for d in _declarations(r):
            syms[d.name()] = d
    for name, v in model.scalars.items():
        d = syms.get(name)
        if d is None:
            continue
        rng = d.range()
        s.add(d() == (z3.BoolVal(bool(v), ctx) if rng.kind() == z3.Z3_BOOL_SORT else z3.BitVecVal(v, rng.size(), ctx)))
    for name, (table, _) in model.arrays.items():
        d = syms.get(name)
        if d is None:
            continue
        arr = d()
        dom, rng = arr.sort().domain().size(), arr.sort().range().size()
        for k, v in table.items():
            s.add(z3.Select(arr, z3.BitVecVal(k, dom, ctx)) == z3.BitVecVal(v, rng, ctx))
    for name, (table, _) in model.funcs.items():
        d = syms.get(name)
        if d is None:
            continue
        for k, v in table.items():
            s.add(d(z3.BitVecVal(k, d.domain(0).size(), ctx)) == z3.BitVecVal(v, d.range().size(), ctx))
    if s.check() != z3.sat:
        return None
    return s.model().translate(z3.main_ctx())


def _declarations(e):
    out, seen, stack = [], set(), [e]
    while stack:
        x = stack.pop()
        if x.get_id() in seen:
            continue
        seen.add(x.get_id())
        if z3.is_app(x) and x.decl().kind() == z3.Z3_OP_UNINTERPRETED:
            out.append(x.decl())
        stack.extend(x.arg(i) for i in range(x.num_args()))
    return out
