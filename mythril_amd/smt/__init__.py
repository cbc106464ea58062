"""Mirror of ``mythril.laser.smt`` over the engine's own term DAG.

Same names, argument meaning and operator overloading as the reference wrappers,
so LASER-style code (and the parity tests, which read like the reference's own
tests) builds exactly the terms LASER would hand to z3:

* ``BitVec`` operators            -> ``mythril/laser/smt/bitvec.py:63-246``
  (``/`` is bvsdiv, ``<``/``>``/``<=``/``>=`` are signed, ``>>`` is bvashr,
  ``==`` zero-pads mixed widths, ``bitvec.py:16-22,183-216``)
* ``If/UGT/UGE/ULT/ULE/Concat/Extract/URem/SRem/UDiv/Sum/BVAddNoOverflow/
  BVMulNoOverflow/BVSubNoUnderflow/LShR`` -> ``bitvec_helper.py:21-214``
  (``UGE``/``ULE`` are ``Or(UGT, ==)``/``Or(ULT, ==)`` exactly as there;
  ``BVAddNoOverflow``/``BVSubNoUnderflow`` expand the way z3's API does;
  ``BVMulNoOverflow`` stays the primitive ``bvumul_noovfl``)
* ``Bool``, ``And/Or/Not/Xor``     -> ``bool.py:14-141``
* ``Array``, ``K``, ``BaseArray``  -> ``array.py:16-63``
* ``Function``                     -> ``function.py:7-25``
* ``symbol_factory``               -> ``smt/__init__.py:83-154``

Differences from the reference, by design: there is no z3, so ``simplify`` only
folds terms whose operands are all literals (enough for the ``.value`` /
``.symbolic`` / ``__bool__`` checks LASER makes on concrete words), and
``Solver``/``Optimize`` (``mythril_amd.solver``) answer ``sat`` by GPU search
or ``unknown`` — they never claim ``unsat``.
"""
from __future__ import annotations

from typing import Any, List, Optional, Set, Union, cast

from . import terms as T
from .fold import fold

Annotations = Set[Any]


class Expression:
    """Base wrapper: ``raw`` term + annotation set (``expression.py:10-55``)."""

    def __init__(self, raw: T.Term, annotations: Optional[Annotations] = None):
        self.raw = raw
        if annotations:
            assert isinstance(annotations, set)
        self._annotations = annotations or set()

    @property
    def annotations(self) -> Annotations:
        return self._annotations

    def annotate(self, annotation: Any) -> None:
        self._annotations.add(annotation)

    def simplify(self) -> None:
        self.raw = fold(self.raw)

    def size(self) -> int:
        return self.raw.width

    def __repr__(self) -> str:
        return repr(self.raw)

    def __hash__(self) -> int:
        return hash(self.raw)

    def get_annotations(self, annotation: Any):
        return [x for x in self.annotations if isinstance(x, annotation)]


def simplify(expression):
    expression.simplify()
    return expression


# ---------------------------------------------------------------------------
# Bool
# ---------------------------------------------------------------------------

class Bool(Expression):
    @property
    def is_false(self) -> bool:
        self.simplify()
        return self.raw.op == "boolconst" and not self.raw.params[0]

    @property
    def is_true(self) -> bool:
        self.simplify()
        return self.raw.op == "boolconst" and bool(self.raw.params[0])

    @property
    def value(self) -> Optional[bool]:
        self.simplify()
        if self.raw.op == "boolconst":
            return bool(self.raw.params[0])
        return None

    def __eq__(self, other) -> "Bool":  # type: ignore[override]
        if isinstance(other, Expression):
            return Bool(T.eq(self.raw, other.raw), self.annotations.union(other.annotations))
        return Bool(T.eq(self.raw, T.BoolVal(bool(other))), set(self.annotations))

    def __ne__(self, other) -> "Bool":  # type: ignore[override]
        return Not(self.__eq__(other))

    def __bool__(self) -> bool:
        v = self.value
        return v if v is not None else False

    def __hash__(self) -> int:
        return hash(self.raw)


def _as_bool(x: Union[Bool, bool]) -> Bool:
    return x if isinstance(x, Bool) else Bool(T.BoolVal(bool(x)))


def And(*args: Union[Bool, bool]) -> Bool:
    lst = [_as_bool(a) for a in args]
    ann: Set = set()
    for a in lst:
        ann |= a.annotations
    return Bool(T.and_(*[a.raw for a in lst]), ann)


def Or(*args: Union[Bool, bool]) -> Bool:
    lst = [_as_bool(a) for a in args]
    ann: Set = set()
    for a in lst:
        ann |= a.annotations
    return Bool(T.or_(*[a.raw for a in lst]), ann)


def Xor(a: Bool, b: Bool) -> Bool:
    return Bool(T.xor_(a.raw, b.raw), a.annotations.union(b.annotations))


def Not(a: Bool) -> Bool:
    return Bool(T.not_(a.raw), set(a.annotations))


def is_false(a: Bool) -> bool:
    return a.raw.op == "boolconst" and not a.raw.params[0]


def is_true(a: Bool) -> bool:
    return a.raw.op == "boolconst" and bool(a.raw.params[0])


# ---------------------------------------------------------------------------
# BitVec
# ---------------------------------------------------------------------------

def _padded(a: T.Term, b: T.Term):
    """``_padded_operation`` (bitvec.py:16-22): zero-extend the narrower side."""
    if a.width == b.width:
        return a, b
    if a.width < b.width:
        a, b = b, a
    b = T.concat(T.BitVecVal(0, a.width - b.width), b)
    return a, b


class BitVec(Expression):
    def size(self) -> int:
        return self.raw.width

    @property
    def symbolic(self) -> bool:
        self.simplify()
        return self.raw.op != "bvconst"

    @property
    def value(self) -> Optional[int]:
        if self.symbolic:
            return None
        return self.raw.params[0]

    def _coerce(self, other) -> "BitVec":
        if isinstance(other, BitVec):
            return other
        return BitVec(T.BitVecVal(int(other), self.size()))

    def _arith(self, op, other) -> "BitVec":
        o = self._coerce(other)
        return BitVec(T.bvbin(op, self.raw, o.raw), self.annotations.union(o.annotations))

    def __add__(self, other):
        return self._arith("bvadd", other)

    def __radd__(self, other):
        return self._coerce(other)._arith("bvadd", self)

    def __sub__(self, other):
        return self._arith("bvsub", other)

    def __rsub__(self, other):
        return self._coerce(other)._arith("bvsub", self)

    def __mul__(self, other):
        return self._arith("bvmul", other)

    def __rmul__(self, other):
        return self._coerce(other)._arith("bvmul", self)

    def __truediv__(self, other):  # z3py '/' on bit-vectors is bvsdiv
        return self._arith("bvsdiv", other)

    def __mod__(self, other):  # z3py '%' on bit-vectors is bvsmod
        return self._arith("bvsmod", other)

    def __and__(self, other):
        return self._arith("bvand", other)

    def __or__(self, other):
        return self._arith("bvor", other)

    def __xor__(self, other):
        return self._arith("bvxor", other)

    def __invert__(self):
        return BitVec(T.bvun("bvnot", self.raw), set(self.annotations))

    def __neg__(self):
        return BitVec(T.bvun("bvneg", self.raw), set(self.annotations))

    def _cmp(self, op, other) -> Bool:
        o = self._coerce(other)
        return Bool(T.bvcmp(op, self.raw, o.raw), self.annotations.union(o.annotations))

    def __lt__(self, other):
        return self._cmp("bvslt", other)

    def __gt__(self, other):
        return self._cmp("bvsgt", other)

    def __le__(self, other):
        return self._cmp("bvsle", other)

    def __ge__(self, other):
        return self._cmp("bvsge", other)

    def __eq__(self, other) -> Bool:  # type: ignore[override]
        if not isinstance(other, BitVec):
            return Bool(T.eq(self.raw, T.BitVecVal(int(other), self.size())), set(self.annotations))
        a, b = _padded(self.raw, other.raw)
        return Bool(T.eq(a, b), self.annotations.union(other.annotations))

    def __ne__(self, other) -> Bool:  # type: ignore[override]
        if not isinstance(other, BitVec):
            return Bool(T.not_(T.eq(self.raw, T.BitVecVal(int(other), self.size()))), set(self.annotations))
        a, b = _padded(self.raw, other.raw)
        return Bool(T.not_(T.eq(a, b)), self.annotations.union(other.annotations))

    def _shift(self, op, other):
        o = self._coerce(other)
        return BitVec(T.bvbin(op, self.raw, o.raw), self.annotations.union(o.annotations))

    def __lshift__(self, other):
        return self._shift("bvshl", other)

    def __rshift__(self, other):  # z3py '>>' is arithmetic
        return self._shift("bvashr", other)

    def __hash__(self) -> int:
        return hash(self.raw)


def _bv(x, width=256) -> BitVec:
    return x if isinstance(x, BitVec) else BitVec(T.BitVecVal(int(x), width))


def _cmp_helper(a: BitVec, b: BitVec, op: str) -> Bool:
    return Bool(T.bvcmp(op, a.raw, b.raw), a.annotations.union(b.annotations))


def _arith_helper(a: BitVec, b: BitVec, op: str) -> BitVec:
    return BitVec(T.bvbin(op, a.raw, b.raw), a.annotations.union(b.annotations))


def LShR(a: BitVec, b: BitVec) -> BitVec:
    return _arith_helper(a, b, "bvlshr")


def If(a: Union[Bool, bool], b: Union[BitVec, int], c: Union[BitVec, int]) -> BitVec:
    a = _as_bool(a)
    b = _bv(b)
    c = _bv(c)
    ann = a.annotations.union(b.annotations).union(c.annotations)
    return BitVec(T.ite(a.raw, b.raw, c.raw), ann)


def UGT(a: BitVec, b: BitVec) -> Bool:
    return _cmp_helper(a, b, "bvugt")


def UGE(a: BitVec, b: BitVec) -> Bool:
    return Or(UGT(a, b), a == b)


def ULT(a: BitVec, b: BitVec) -> Bool:
    return _cmp_helper(a, b, "bvult")


def ULE(a: BitVec, b: BitVec) -> Bool:
    return Or(ULT(a, b), a == b)


def Concat(*args) -> BitVec:
    bvs = args[0] if len(args) == 1 and isinstance(args[0], list) else list(args)
    ann: Set = set()
    for b in bvs:
        ann |= b.annotations
    return BitVec(T.concat(*[b.raw for b in bvs]), ann)


def Extract(high: int, low: int, bv: BitVec) -> BitVec:
    return BitVec(T.extract(high, low, bv.raw), set(bv.annotations))


def URem(a: BitVec, b: BitVec) -> BitVec:
    return _arith_helper(a, b, "bvurem")


def SRem(a: BitVec, b: BitVec) -> BitVec:
    return _arith_helper(a, b, "bvsrem")


def UDiv(a: BitVec, b: BitVec) -> BitVec:
    return _arith_helper(a, b, "bvudiv")


def Sum(*args: BitVec) -> BitVec:
    ann: Set = set()
    acc = args[0].raw
    for b in args:
        ann |= b.annotations
    for b in args[1:]:
        acc = T.bvbin("bvadd", acc, b.raw)
    return BitVec(acc, ann)


def BVAddNoOverflow(a, b, signed: bool) -> Bool:
    """z3's ``Z3_mk_bvadd_no_overflow`` expansion (unsigned case): the carry-out
    bit of the (w+1)-bit sum is zero.  Signed form is not emitted by LASER."""
    a, b = _bv(a), _bv(b)
    if signed:
        raise NotImplementedError("signed BVAddNoOverflow is not emitted by LASER")
    w = a.size()
    s = T.bvbin("bvadd", T.zero_extend(1, a.raw), T.zero_extend(1, b.raw))
    return Bool(T.eq(T.extract(w, w, s), T.BitVecVal(0, 1)))


def BVMulNoOverflow(a, b, signed: bool) -> Bool:
    """``bvumul_noovfl`` primitive (bitvec_helper.py:183-196)."""
    a, b = _bv(a), _bv(b)
    if signed:
        raise NotImplementedError("signed BVMulNoOverflow is not emitted by LASER")
    return Bool(T.bvcmp("bvumul_noovfl", a.raw, b.raw))


def BVSubNoUnderflow(a, b, signed: bool) -> Bool:
    """z3's ``Z3_mk_bvsub_no_underflow`` (unsigned): ``bvule(b, a)``."""
    a, b = _bv(a), _bv(b)
    if signed:
        raise NotImplementedError("signed BVSubNoUnderflow is not emitted by LASER")
    return Bool(T.bvcmp("bvule", b.raw, a.raw))


# ---------------------------------------------------------------------------
# Arrays and functions
# ---------------------------------------------------------------------------

class BaseArray:
    raw: T.Term

    def __getitem__(self, item: BitVec) -> BitVec:
        if isinstance(item, slice):
            raise ValueError("Instance of BaseArray, does not support getitem with slices")
        return BitVec(T.select(self.raw, item.raw))

    def __setitem__(self, key: BitVec, value: BitVec) -> None:
        if isinstance(value, Bool):
            value = If(value, 1, 0)
        self.raw = T.store(self.raw, key.raw, value.raw)


class Array(BaseArray):
    def __init__(self, name: str, domain: int, value_range: int):
        self.domain = domain
        self.range = value_range
        self.raw = T.ArrayVar(name, domain, value_range)


class K(BaseArray):
    def __init__(self, domain: int, value_range: int, value: int):
        self.domain = domain
        self.range = value_range
        self.value = T.BitVecVal(value, value_range)
        self.raw = T.ConstArray(domain, self.value)


class Function:
    def __init__(self, name: str, domain: int, value_range: int):
        self.domain = domain
        self.range = value_range
        self.raw = T.FuncDecl(name, domain, value_range)

    def __call__(self, item: BitVec) -> BitVec:
        return BitVec(T.app(self.raw, item.raw), set(item.annotations))


# ---------------------------------------------------------------------------
# symbol factory
# ---------------------------------------------------------------------------

class _SmtSymbolFactory:
    @staticmethod
    def Bool(value: bool, annotations: Annotations = None) -> Bool:
        return Bool(T.BoolVal(value), annotations)

    @staticmethod
    def BoolSym(name: str, annotations: Annotations = None) -> Bool:
        return Bool(T.BoolVar(name), annotations)

    @staticmethod
    def BitVecVal(value: int, size: int, annotations: Annotations = None) -> BitVec:
        return BitVec(T.BitVecVal(value, size), annotations)

    @staticmethod
    def BitVecSym(name: str, size: int, annotations: Annotations = None) -> BitVec:
        return BitVec(T.BitVecVar(name, size), annotations)


symbol_factory = _SmtSymbolFactory()

__all__ = [
    "Expression", "simplify", "Bool", "And", "Or", "Xor", "Not", "is_true", "is_false",
    "BitVec", "If", "UGT", "UGE", "ULT", "ULE", "Concat", "Extract", "URem", "SRem",
    "UDiv", "Sum", "BVAddNoOverflow", "BVMulNoOverflow", "BVSubNoUnderflow", "LShR",
    "BaseArray", "Array", "K", "Function", "symbol_factory",
]
