"""Hash-consed term DAG: the host-side AST that the ``mythril_amd.smt`` mirror builds.

In the reference every ``BitVec``/``Bool``/``Array``/``Function`` wraps a z3 AST
(``mythril/laser/smt/expression.py:10-33``).  z3 is not part of this build, so the
mirror wraps a :class:`Term` instead.  Terms are structurally hash-consed (the same
as z3's ``get_id()`` sharing), immutable, and carry only what the SSA flattener
(``mythril_amd/ssa.py``) needs.  The operator vocabulary is exactly the set of z3
constructs LASER emits, plus two EVM extensions used by concrete
replay programs: ``keccak256`` (real Keccak-256 of the big-endian bytes of a
value) and ``bvexp`` (EVM EXP, mod 2^w).

Sorts
-----
* ``("bv", w)``   bit-vector of width ``w``
* ``("bool",)``   boolean (evaluated as a 1-bit value by the engine)
* ``("array", d, r)`` array BitVec(d) -> BitVec(r)
"""
from __future__ import annotations

import itertools
import threading
import weakref
from typing import Iterable, Optional, Tuple

BOOL = ("bool",)

# Operators and the sort discipline the builder enforces.
BV_BINARY = frozenset(
    "bvadd bvsub bvmul bvudiv bvurem bvsdiv bvsrem bvsmod bvand bvor bvxor "
    "bvshl bvlshr bvashr bvexp".split()
)
BV_UNARY = frozenset(("bvnot", "bvneg"))
BV_COMPARE = frozenset(
    "bvult bvule bvugt bvuge bvslt bvsle bvsgt bvsge bvumul_noovfl".split()
)
BOOL_NARY = frozenset(("and", "or"))

_lock = threading.Lock()
_table: "weakref.WeakValueDictionary[tuple, Term]" = weakref.WeakValueDictionary()
_ids = itertools.count(1)


class Term:
    """One node of the DAG.  Construct through :func:`mk`, never directly."""

    __slots__ = ("op", "sort", "args", "params", "id", "_key", "__weakref__")

    def __init__(self, op, sort, args, params, key):
        self.op = op
        self.sort = sort
        self.args = args
        self.params = params
        self.id = next(_ids)
        self._key = key

    # -- sort helpers -------------------------------------------------
    @property
    def is_bool(self) -> bool:
        return self.sort[0] == "bool"

    @property
    def is_bv(self) -> bool:
        return self.sort[0] == "bv"

    @property
    def is_array(self) -> bool:
        return self.sort[0] == "array"

    @property
    def width(self) -> int:
        """Bit width of a bit-vector (1 for a Bool)."""
        if self.sort[0] == "bv":
            return self.sort[1]
        if self.sort[0] == "bool":
            return 1
        raise TypeError("array terms have no width")

    def size(self) -> int:
        return self.width

    def __hash__(self):
        return self.id

    def __eq__(self, other):  # identity == structural equality (hash-consed)
        return self is other

    def __repr__(self):
        return to_sexpr(self, depth=3)


def mk(op: str, sort: tuple, args: Tuple["Term", ...] = (), params: tuple = ()) -> Term:
    """Return the unique term for (op, sort, args, params)."""
    key = (op, sort, tuple(a.id for a in args), params)
    with _lock:
        t = _table.get(key)
        if t is None:
            t = Term(op, sort, tuple(args), params, key)
            _table[key] = t
        return t


# ----------------------------------------------------------------------------
# constructors (the z3 API subset LASER uses)
# ----------------------------------------------------------------------------

def bv_sort(w: int) -> tuple:
    if w <= 0:
        raise ValueError("bit-vector width must be positive")
    return ("bv", int(w))


def BitVecVal(value: int, w: int) -> Term:
    return mk("bvconst", bv_sort(w), (), (int(value) % (1 << w),))


def BitVecVar(name: str, w: int) -> Term:
    return mk("bvvar", bv_sort(w), (), (str(name),))


def BoolVal(b: bool) -> Term:
    return mk("boolconst", BOOL, (), (bool(b),))


def BoolVar(name: str) -> Term:
    return mk("boolvar", BOOL, (), (str(name),))


def _same_bv(a: Term, b: Term, op: str):
    if not (a.is_bv and b.is_bv):
        raise TypeError(f"{op}: bit-vector operands required")
    if a.width != b.width:
        raise TypeError(f"{op}: width mismatch {a.width} vs {b.width}")


def bvbin(op: str, a: Term, b: Term) -> Term:
    assert op in BV_BINARY, op
    _same_bv(a, b, op)
    return mk(op, a.sort, (a, b))


def bvun(op: str, a: Term) -> Term:
    assert op in BV_UNARY, op
    if not a.is_bv:
        raise TypeError(op)
    return mk(op, a.sort, (a,))


def bvcmp(op: str, a: Term, b: Term) -> Term:
    assert op in BV_COMPARE, op
    _same_bv(a, b, op)
    return mk(op, BOOL, (a, b))


def eq(a: Term, b: Term) -> Term:
    if a.sort != b.sort:
        raise TypeError(f"eq: sort mismatch {a.sort} vs {b.sort}")
    return mk("eq", BOOL, (a, b))


def concat(*parts: Term) -> Term:
    """z3.Concat: first argument is the most significant part."""
    if len(parts) == 1:
        return parts[0]
    for p in parts:
        if not p.is_bv:
            raise TypeError("concat of non bit-vector")
    # left fold into binary nodes: ((a ++ b) ++ c)
    acc = parts[0]
    for p in parts[1:]:
        acc = mk("concat", bv_sort(acc.width + p.width), (acc, p))
    return acc


def extract(hi: int, lo: int, a: Term) -> Term:
    if not a.is_bv or not (0 <= lo <= hi < a.width):
        raise ValueError(f"extract({hi},{lo}) of width {a.width if a.is_bv else a.sort}")
    return mk("extract", bv_sort(hi - lo + 1), (a,), (hi, lo))


def zero_extend(k: int, a: Term) -> Term:
    if k == 0:
        return a
    return mk("zero_extend", bv_sort(a.width + k), (a,), (k,))


def sign_extend(k: int, a: Term) -> Term:
    if k == 0:
        return a
    return mk("sign_extend", bv_sort(a.width + k), (a,), (k,))


def ite(c: Term, a: Term, b: Term) -> Term:
    if not c.is_bool:
        raise TypeError("ite condition must be Bool")
    if a.sort != b.sort:
        raise TypeError(f"ite: branch sorts differ {a.sort} vs {b.sort}")
    return mk("ite", a.sort, (c, a, b))


def and_(*args: Term) -> Term:
    args = tuple(args)
    for a in args:
        if not a.is_bool:
            raise TypeError("And of non-Bool")
    if len(args) == 0:
        return BoolVal(True)
    if len(args) == 1:
        return args[0]
    return mk("and", BOOL, args)


def or_(*args: Term) -> Term:
    args = tuple(args)
    for a in args:
        if not a.is_bool:
            raise TypeError("Or of non-Bool")
    if len(args) == 0:
        return BoolVal(False)
    if len(args) == 1:
        return args[0]
    return mk("or", BOOL, args)


def not_(a: Term) -> Term:
    if not a.is_bool:
        raise TypeError("Not of non-Bool")
    return mk("not", BOOL, (a,))


def xor_(a: Term, b: Term) -> Term:
    if not (a.is_bool and b.is_bool):
        raise TypeError("Xor of non-Bool")
    return mk("xor", BOOL, (a, b))


# arrays ------------------------------------------------------------------

def ArrayVar(name: str, dom: int, rng: int) -> Term:
    return mk("array_var", ("array", int(dom), int(rng)), (), (str(name),))


def ConstArray(dom: int, value: Term) -> Term:
    if not value.is_bv:
        raise TypeError("K() value must be a bit-vector")
    return mk("const_array", ("array", int(dom), value.width), (value,))


def store(arr: Term, idx: Term, val: Term) -> Term:
    if not arr.is_array:
        raise TypeError("Store on non-array")
    _, d, r = arr.sort
    if not (idx.is_bv and idx.width == d and val.is_bv and val.width == r):
        raise TypeError("Store: index/value sort mismatch")
    return mk("store", arr.sort, (arr, idx, val))


def select(arr: Term, idx: Term) -> Term:
    if not arr.is_array:
        raise TypeError("Select on non-array")
    _, d, r = arr.sort
    if not (idx.is_bv and idx.width == d):
        raise TypeError("Select: index sort mismatch")
    return mk("select", bv_sort(r), (arr, idx))


# uninterpreted functions ------------------------------------------------

class FuncDecl:
    """An uninterpreted function declaration f: BitVec(dom) -> BitVec(rng)."""

    __slots__ = ("name", "dom", "rng")

    def __init__(self, name: str, dom: int, rng: int):
        self.name, self.dom, self.rng = str(name), int(dom), int(rng)

    def key(self):
        return (self.name, self.dom, self.rng)

    def __eq__(self, other):
        return isinstance(other, FuncDecl) and self.key() == other.key()

    def __hash__(self):
        return hash(self.key())

    def __call__(self, arg: Term) -> Term:
        return app(self, arg)

    def __repr__(self):
        return f"FuncDecl({self.name}: bv{self.dom} -> bv{self.rng})"


def app(f: FuncDecl, arg: Term) -> Term:
    if not (arg.is_bv and arg.width == f.dom):
        raise TypeError(f"{f.name}: argument width {arg.width if arg.is_bv else arg.sort} != {f.dom}")
    return mk("app", bv_sort(f.rng), (arg,), f.key())


# EVM extensions -----------------------------------------------------------

def keccak256(data: Term) -> Term:
    """Concrete Keccak-256 of the ``width/8`` big-endian bytes of ``data``."""
    if not data.is_bv or data.width % 8:
        raise TypeError("keccak256 needs a byte-aligned bit-vector")
    return mk("keccak256", bv_sort(256), (data,))


def keccak256_empty() -> Term:
    return mk("keccak256", bv_sort(256), (), ("empty",))


def bvexp(a: Term, b: Term) -> Term:
    return bvbin("bvexp", a, b)


# ----------------------------------------------------------------------------
# traversal helpers
# ----------------------------------------------------------------------------

def postorder(roots: Iterable[Term], skip=None):
    """Yield every distinct term reachable from ``roots`` children-first.  Terms
    whose id is in ``skip`` (a set or dict) are neither yielded nor expanded."""
    seen = set(skip) if skip is not None else set()
    out = []
    stack = [(r, False) for r in reversed(list(roots))]
    while stack:
        t, done = stack.pop()
        if done:
            out.append(t)
            continue
        if t.id in seen:
            continue
        seen.add(t.id)
        stack.append((t, True))
        for a in reversed(t.args):
            if a.id not in seen:
                stack.append((a, False))
    # duplicates can appear when a node is pushed twice before being visited
    res, emitted = [], set()
    for t in out:
        if t.id not in emitted:
            emitted.add(t.id)
            res.append(t)
    return res


def free_symbols(roots: Iterable[Term]):
    """Names of scalar variables, arrays and functions a set of terms depends on."""
    out = set()
    for t in postorder(roots):
        if t.op in ("bvvar", "boolvar", "array_var"):
            out.add(t.params[0])
        elif t.op == "app":
            out.add(t.params[0])
    return out


def is_const(t: Term) -> bool:
    return t.op in ("bvconst", "boolconst")


def const_value(t: Term) -> Optional[int]:
    if t.op == "bvconst":
        return t.params[0]
    if t.op == "boolconst":
        return int(t.params[0])
    return None


def to_sexpr(t: Term, depth: int = 1 << 30) -> str:
    if t.op == "bvconst":
        return f"#x{t.params[0]:0{max(1, (t.width + 3) // 4)}x}" if t.width % 4 == 0 else f"(_ bv{t.params[0]} {t.width})"
    if t.op == "boolconst":
        return "true" if t.params[0] else "false"
    if t.op in ("bvvar", "boolvar", "array_var"):
        return str(t.params[0])
    if depth <= 0:
        return "…"
    head = t.op
    if t.op == "extract":
        head = f"(_ extract {t.params[0]} {t.params[1]})"
    elif t.op in ("zero_extend", "sign_extend"):
        head = f"(_ {t.op} {t.params[0]})"
    elif t.op == "app":
        head = t.params[0]
    elif t.op == "const_array":
        head = "(as const)"
    inner = " ".join(to_sexpr(a, depth - 1) for a in t.args)
    return f"({head} {inner})" if inner else f"({head})"
