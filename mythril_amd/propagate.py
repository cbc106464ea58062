"""Constraint propagation onto candidate coordinates (search-space shaping).

Random candidates almost never satisfy the equalities LASER queries are built
from — a 4-byte selector match alone is a 2^-32 event.  Before searching, this
pass walks the conjunction (the ``Bool`` tuple ``get_model`` receives,
``mythril/support/model.py:36-39``) and pushes simple facts down to the
coordinates that carry them:

* ``x == c`` through ``Concat``/``Extract``/``ZeroExt``/``UDiv`` by ``2^k`` /
  ``And`` with a low mask / ``+``/``-``/``^`` a literal / ``If(c, x, 0)`` —
  the solc dispatcher's ``DIV(CALLDATALOAD(0), 2^224) & 0xffffffff == sel``
  (``instructions.py:480-494, 716-740``) becomes four fixed calldata bytes plus
  ``size > i`` for each byte read (``calldata.py:226-231``);
* ``Or(x == c1, x == c2, ...)`` -> a dictionary (the actor disjunction,
  ``transaction/symbolic.py:165-167``);
* unsigned / signed bounds against literals, through ``x - c`` (with wrap) ->
  an interval union (``If(ULT(size - 4, 64), 1, 0) == 0`` -> size >= 68);
* ``If(c, 1, 0) != 0`` / ``== 0`` -> ``c`` / ``Not(c)`` (``pop_bitvec``, ``util.py:78-83``);
* ``URem(x, 2^k) == 0`` -> low k bits fixed to zero (the keccak ``mod 64`` condition).

The result only changes WHICH candidates are drawn (generator specs); every
candidate is still evaluated in full by the kernel, so a wrong guess costs hits,
never correctness.  Facts that conflict with an earlier one are dropped.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from . import ssa
from .smt import terms as T


def _mask(w):
    return (1 << w) - 1


class Domain:
    """Refinement of one coordinate: fixed bits, a union of intervals, a choice set."""

    __slots__ = ("width", "fmask", "fval", "intervals", "choices")

    def __init__(self, width: int):
        self.width = width
        self.fmask = 0
        self.fval = 0
        self.intervals: Optional[List[Tuple[int, int]]] = None  # inclusive, sorted, disjoint
        self.choices: Optional[List[int]] = None

    def fix_bits(self, lo: int, nbits: int, value: int) -> bool:
        m = _mask(nbits) << lo
        v = (value & _mask(nbits)) << lo
        if (self.fmask & m) and ((self.fval ^ v) & self.fmask & m):
            return False  # conflicting fact: keep the first
        self.fmask |= m
        self.fval = (self.fval & ~m) | v
        return True

    def restrict(self, ivs: List[Tuple[int, int]]) -> bool:
        ivs = _norm(ivs)
        new = ivs if self.intervals is None else _intersect(self.intervals, ivs)
        if not new:
            return False
        self.intervals = new
        return True

    def choose(self, values: Sequence[int]) -> bool:
        vals = sorted(set(v & _mask(self.width) for v in values))
        if self.choices is not None:
            vals = [v for v in vals if v in self.choices]
        if not vals:
            return False
        self.choices = vals
        return True

    def admissible(self, v: int) -> bool:
        if (v & self.fmask) != self.fval:
            return False
        if self.intervals is not None and not any(a <= v <= b for a, b in self.intervals):
            return False
        return True


def _norm(ivs):
    ivs = sorted((a, b) for a, b in ivs if a <= b)
    out = []
    for a, b in ivs:
        if out and a <= out[-1][1] + 1:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _intersect(x, y):
    out = []
    for a, b in x:
        for c, d in y:
            lo, hi = max(a, c), min(b, d)
            if lo <= hi:
                out.append((lo, hi))
    return _norm(out)


def _shift(ivs, c, w):
    """{v + c mod 2^w : v in ivs}"""
    m = 1 << w
    out = []
    for a, b in ivs:
        a2, b2 = (a + c) % m, (b + c) % m
        if b - a >= m - 1:
            return [(0, m - 1)]
        if a2 <= b2:
            out.append((a2, b2))
        else:
            out += [(a2, m - 1), (0, b2)]
    return _norm(out)


class Propagator:
    def __init__(self, P: ssa.Program):
        self.P = P
        self.dom: Dict[int, Domain] = {}
        self.term_ivs: Dict[int, List[Tuple[int, int]]] = {}  # interval facts on non-coordinate terms
        # term id -> coordinate index, for terms that ARE a coordinate's value
        self.coord_of: Dict[int, int] = {}
        self.base_read_of: Dict[int, int] = {}
        # term id -> (AUX coordinate, bit offset): a calldata byte that is a slice of an AUX word
        self.slice_of: Dict[int, Tuple[int, int]] = {}
        self.hints: List[T.Term] = []  # terms a symbolic comparison wants small
        for c in P.coords:
            t = c.term
            if c.kind == ssa.COORD_SCALAR:
                self.coord_of[t.id] = c.index
            elif c.kind == ssa.COORD_AUX:
                continue
            elif c.kind == ssa.COORD_ARRAY_SITE:
                if c.index in P.aux_slice:  # the site's value is bits of an AUX word (ssa.calldata_window)
                    self.slice_of[t.id] = P.aux_slice[c.index]
                elif t.args[0].op == "array_var":  # a store chain would override the value
                    self.coord_of[t.id] = c.index
                else:  # the base read a store-chain select falls through to when no index matches
                    self.base_read_of[t.id] = c.index
            else:
                if P.nodes[c.node][7] == ssa.MG_NONE:  # lazily-defaulted sites are not free
                    self.coord_of[t.id] = c.index

    def d(self, c: int) -> Domain:
        if c not in self.dom:
            self.dom[c] = Domain(self.P.coords[c].width)
        return self.dom[c]

    # -- bit-vector facts -------------------------------------------
    def eq_bits(self, t: T.Term, lo: int, n: int, value: int, depth=0) -> bool:
        """Assume bits [lo, lo+n) of t equal `value`."""
        if depth > 64 or n <= 0:
            return False
        w = t.width
        if lo >= w:
            return value == 0
        if lo + n > w:
            # bits beyond the width are zero
            if value >> (w - lo):
                return False
            n = w - lo
        value &= _mask(n)
        sl = self.slice_of.get(t.id)
        if sl is not None:
            return self.d(sl[0]).fix_bits(sl[1] + lo, n, value)
        c = self.coord_of.get(t.id)
        if c is None:
            c = self.base_read_of.get(t.id)
        if c is not None:
            return self.d(c).fix_bits(lo, n, value)
        op = t.op
        if op == "bvconst":
            return ((t.params[0] >> lo) & _mask(n)) == value
        if op == "concat":
            a, b = t.args
            wb = b.width
            ok = True
            if lo < wb:
                nb = min(n, wb - lo)
                ok &= self.eq_bits(b, lo, nb, value & _mask(nb), depth + 1)
            if lo + n > wb:
                la = max(0, lo - wb)
                skip = max(0, wb - lo)
                ok &= self.eq_bits(a, la, n - skip, value >> skip, depth + 1)
            return ok
        if op == "extract":
            hi_, lo_ = t.params
            return self.eq_bits(t.args[0], lo_ + lo, n, value, depth + 1)
        if op == "zero_extend":
            return self.eq_bits(t.args[0], lo, n, value, depth + 1)
        if op == "bvudiv":
            k = _pow2(t.args[1])
            if k is not None:
                return self.eq_bits(t.args[0], lo + k, n, value, depth + 1)
        if op == "bvand":
            for x, m in ((t.args[0], t.args[1]), (t.args[1], t.args[0])):
                if m.op == "bvconst":
                    mv = (m.params[0] >> lo) & _mask(n)
                    if value & ~mv:
                        return False  # a masked-off bit would have to be 1
                    # every run of mask ones carries the requested bits to x
                    ok, i = True, 0
                    while i < n:
                        if not (mv >> i) & 1:
                            i += 1
                            continue
                        j = i
                        while j < n and (mv >> j) & 1:
                            j += 1
                        ok &= self.eq_bits(x, lo + i, j - i, value >> i, depth + 1)
                        i = j
                    return ok
        if op == "ite":
            cnd, x, y = t.args
            xv = (x.params[0] >> lo) & _mask(n) if x.op == "bvconst" else None
            yv = (y.params[0] >> lo) & _mask(n) if y.op == "bvconst" else None
            # If(c, x, k) == v with k != v forces c and x == v (a calldata byte read
            # If(i < size, calldata[i], 0) == nonzero); with k == v, constraining the
            # other branch to v satisfies the equality whatever c is
            if yv is not None and yv != value:
                return self.assume(cnd, True, depth + 1) and self.eq_bits(x, lo, n, value, depth + 1)
            if xv is not None and xv != value:
                return self.assume(cnd, False, depth + 1) and self.eq_bits(y, lo, n, value, depth + 1)
            if yv is not None and x.op != "bvconst":
                return self.eq_bits(x, lo, n, value, depth + 1)
            if xv is not None and y.op != "bvconst":
                return self.eq_bits(y, lo, n, value, depth + 1)
            if xv is None and yv is None:
                return self.eq_bits(x, lo, n, value, depth + 1) | self.eq_bits(y, lo, n, value, depth + 1)
            return False
        if lo == 0 and n == w:
            if op in ("bvadd", "bvsub", "bvxor"):
                a, b = t.args
                if b.op == "bvconst" or (a.op == "bvconst" and op != "bvsub"):
                    x, k = (a, b.params[0]) if b.op == "bvconst" else (b, a.params[0])
                    inv = {"bvadd": (value - k), "bvsub": (value + k), "bvxor": value ^ k}[op]
                    return self.eq_bits(x, 0, w, inv & _mask(w), depth + 1)
            if op == "bvurem":
                k = _pow2(t.args[1])
                if k is not None and value >> k == 0:
                    return self.eq_bits(t.args[0], 0, k, value, depth + 1)
        return False

    def bound(self, t: T.Term, ivs: List[Tuple[int, int]], depth=0) -> bool:
        """Assume t (unsigned) lies in the interval union."""
        c = self.coord_of.get(t.id)
        if c is None:
            c = self.base_read_of.get(t.id)
        w = t.width
        if c is not None:
            return self.d(c).restrict(ivs)
        if depth > 32:
            return False
        if t.op in ("bvadd", "bvsub"):
            a, b = t.args
            if b.op == "bvconst":
                k = b.params[0]
                return self.bound(a, _shift(ivs, (-k if t.op == "bvadd" else k), w), depth + 1)
        if t.op == "zero_extend":
            inner = _intersect(ivs, [(0, _mask(t.args[0].width))])
            return bool(inner) and self.bound(t.args[0], inner, depth + 1)
        if t.op == "ite":
            # bound both arms: the fact then holds whichever way the condition goes
            # (yetNeeded = If(pending == 0, m_required, pending) <= 1)
            ok = False
            for arm in t.args[1:]:
                if arm.op != "bvconst":
                    ok |= self.bound(arm, ivs, depth + 1)
            return ok
        # any other term: intersect with what earlier facts said about it, and fix the
        # high bits every admissible value shares (a calldata word bounded to [1, 1] by
        # a loop's two JUMPI conditions becomes 32 fixed bytes)
        prev = self.term_ivs.get(t.id)
        ivs = _norm(ivs) if prev is None else _intersect(prev, ivs)
        if not ivs:
            return False
        self.term_ivs[t.id] = ivs
        lo, hi = ivs[0][0], ivs[-1][1]
        k = (lo ^ hi).bit_length()
        return k < w and self.eq_bits(t, k, w - k, lo >> k, depth + 1)

    # -- boolean facts ----------------------------------------------
    def assume(self, b: T.Term, truth: bool, depth=0) -> bool:
        if depth > 64:
            return False
        op = b.op
        if op == "boolconst":
            return bool(b.params[0]) == truth
        if op == "not":
            return self.assume(b.args[0], not truth, depth + 1)
        if op == "and" and truth or op == "or" and not truth:
            ok = True
            for a in b.args:
                ok &= self.assume(a, truth, depth + 1)
            return ok
        if op == "or" and truth:
            live = [a for a in b.args if not (a.op == "boolconst" and not a.params[0])]
            if len(live) == 1:
                return self.assume(live[0], True, depth + 1)
            # Or(x < y, x == y): the mirror's UGE/ULE (bitvec_helper.py:54-80)
            if len(live) == 2:
                cmp_, eq_ = (live[0], live[1]) if live[1].op == "eq" else (live[1], live[0])
                nonstrict = {"bvult": "bvule", "bvugt": "bvuge", "bvslt": "bvsle", "bvsgt": "bvsge"}
                if eq_.op == "eq" and cmp_.op in nonstrict and {x.id for x in cmp_.args} == {x.id for x in eq_.args}:
                    return self._cmp(nonstrict[cmp_.op], cmp_.args[0], cmp_.args[1], True, depth)
            # Or(x == c1, x == c2, ...) over one coordinate -> choices
            target, vals = None, []
            for a in live:
                if a.op != "eq":
                    return False
                x, k = a.args
                if x.op == "bvconst":
                    x, k = k, x
                if k.op != "bvconst" or (target is not None and x.id != target.id):
                    return False
                target = x
                vals.append(k.params[0])
            c = self.coord_of.get(target.id) if target is not None else None
            return c is not None and self.d(c).choose(vals)
        if op == "eq":
            x, y = b.args
            if x.is_bool:
                if y.op == "boolconst":
                    return self.assume(x, truth == bool(y.params[0]), depth + 1)
                if x.op == "boolconst":
                    return self.assume(y, truth == bool(x.params[0]), depth + 1)
                return False
            if x.op == "bvconst":
                x, y = y, x
            if y.op != "bvconst":
                return False
            v = y.params[0]
            if truth:
                return self.eq_bits(x, 0, x.width, v, depth + 1)
            # x != v with x = If(c, k1, k2) (pop_bitvec / ISZERO shapes)
            if x.op == "ite" and x.args[1].op == "bvconst" and x.args[2].op == "bvconst":
                k1, k2 = x.args[1].params[0], x.args[2].params[0]
                if k1 == v and k2 != v:
                    return self.assume(x.args[0], False, depth + 1)
                if k2 == v and k1 != v:
                    return self.assume(x.args[0], True, depth + 1)
            return False
        if op in ("bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge"):
            return self._cmp(op, b.args[0], b.args[1], truth, depth)
        return False

    def _cmp(self, op, a, b, truth, depth) -> bool:
        # normalise to  x OP k  with k literal
        flip = {"bvult": "bvugt", "bvule": "bvuge", "bvugt": "bvult", "bvuge": "bvule",
                "bvslt": "bvsgt", "bvsle": "bvsge", "bvsgt": "bvslt", "bvsge": "bvsle"}
        if a.op == "bvconst" and b.op != "bvconst":
            a, b, op = b, a, flip[op]
        if b.op != "bvconst":
            # symbolic on both sides: hint that the smaller side is small, applied after
            # every literal fact (so it never displaces one): newRequired <= m_numOwners
            if not truth:
                op = {"bvult": "bvuge", "bvule": "bvugt", "bvugt": "bvule", "bvuge": "bvult",
                      "bvslt": "bvsge", "bvsle": "bvsgt", "bvsgt": "bvsle", "bvsge": "bvslt"}[op]
            small = a if op in ("bvult", "bvule", "bvslt", "bvsle") else b
            self.hints.append(small)
            return False
        if not truth:
            op = {"bvult": "bvuge", "bvule": "bvugt", "bvugt": "bvule", "bvuge": "bvult",
                  "bvslt": "bvsge", "bvsle": "bvsgt", "bvsgt": "bvsle", "bvsge": "bvslt"}[op]
        w = a.width
        k = b.params[0]
        M = _mask(w)
        if op.startswith("bvs"):
            # signed: map to unsigned intervals of the two's-complement encoding
            ks = k - (1 << w) if k >> (w - 1) else k
            lo_s, hi_s = -(1 << (w - 1)), (1 << (w - 1)) - 1
            rng = {"bvslt": (lo_s, ks - 1), "bvsle": (lo_s, ks), "bvsgt": (ks + 1, hi_s), "bvsge": (ks, hi_s)}[op]
            a_, b_ = rng
            if a_ > b_:
                return False
            ivs = []
            for x0, x1 in ((a_, min(b_, -1)), (max(a_, 0), b_)):
                if x0 <= x1:
                    ivs.append((x0 % (1 << w), x1 % (1 << w)))
        else:
            rng = {"bvult": (0, k - 1), "bvule": (0, k), "bvugt": (k + 1, M), "bvuge": (k, M)}[op]
            if rng[0] > rng[1]:
                return False
            ivs = [rng]
        return self.bound(a, ivs, depth + 1)


def _pow2(t: T.Term) -> Optional[int]:
    if t.op != "bvconst":
        return None
    v = t.params[0]
    if v and not (v & (v - 1)):
        return v.bit_length() - 1
    return None


def propagate(P: ssa.Program, roots: Sequence[T.Term]) -> Dict[int, Domain]:
    pr = Propagator(P)
    for r in roots:
        pr.assume(r, True)
    for t in pr.hints:
        if t.op != "bvconst" and t.width > 8:
            pr.bound(t, [(0, 255)])
    return pr.dom
