"""Flatten a path-constraint DAG into the engine's SSA program (format v1,
``include/mythgpu.h``).

This is step (1) of the north-star pipeline: the constraint tuple that
``get_model`` (``mythril/support/model.py:15-49``) would ``Optimize.add`` to z3 is
hash-consed (terms are already shared, like z3 ``get_id()``), topologically
ordered and emitted as fixed 8-word nodes.  Every operand index refers to an
earlier node, so the native loader can lower and register-allocate in one pass.

Candidate coordinates
---------------------
* every scalar variable (``BitVec``/``Bool`` symbol) is one coordinate;
* every ``Select`` whose store chain bottoms out at an array *variable*
  (``Storage``, ``balance``, ``<tx>_calldata``; ``calldata.py:215-216``,
  ``account.py:62``, ``world_state.py:33``) is an array *site* with its own
  coordinate;
* every uninterpreted-function application (``keccak256_<n>`` and its inverse,
  ``keccak_function_manager.py:59-72``) is a UF site with its own coordinate.

The engine canonicalises sites per lane: a site whose index/argument VALUE equals
an earlier site's of the same array/function returns that site's value
(Ackermann consistency), so every candidate is a genuine finite z3 model
(tables + ``else``) — see ``model_from_sites`` below.

Inverse-UF sites ``inv(f(x))`` get a *lazy default* of ``x`` (the value the
keccak side condition ``inv(f(x)) == x``, ``keccak_function_manager.py:138-149``,
asks for); the model is still an honest table entry.
"""
from __future__ import annotations

import struct
from typing import Dict, Iterable, List, Optional, Sequence

from .smt import terms as T

MG_MAGIC = 0x3150474D
MG_VERSION = 2
MG_NONE = 0xFFFFFFFF
MG_MAX_WIDTH = 32768

# opcode numbers — must equal enum mg_op in include/mythgpu.h (checked by tests)
OPS = {
    "CONST": 0, "VAR": 1, "ADD": 2, "SUB": 3, "MUL": 4, "UDIV": 5, "UREM": 6, "SDIV": 7,
    "SREM": 8, "SMOD": 9, "AND": 10, "OR": 11, "XOR": 12, "NOT": 13, "NEG": 14, "SHL": 15,
    "LSHR": 16, "ASHR": 17, "CONCAT": 18, "EXTRACT": 19, "ZEXT": 20, "SEXT": 21, "ITE": 22,
    "EQ": 23, "ULT": 24, "ULE": 25, "SLT": 26, "SLE": 27, "UMUL_NOOVF": 28, "ARR_VAR": 29,
    "ARR_K": 30, "ARR_STORE": 31, "SELECT": 32, "UFAPP": 33, "KECCAK": 34, "EXP": 35,
}
COORD_SCALAR, COORD_ARRAY_SITE, COORD_UF_SITE, COORD_AUX = 0, 1, 2, 3
TABLE_ARRAY, TABLE_UF = 0, 1

_BIN = {
    "bvadd": "ADD", "bvsub": "SUB", "bvmul": "MUL", "bvudiv": "UDIV", "bvurem": "UREM",
    "bvsdiv": "SDIV", "bvsrem": "SREM", "bvsmod": "SMOD", "bvand": "AND", "bvor": "OR",
    "bvxor": "XOR", "bvshl": "SHL", "bvlshr": "LSHR", "bvashr": "ASHR", "bvexp": "EXP",
    "bvult": "ULT", "bvule": "ULE", "bvslt": "SLT", "bvsle": "SLE",
    "bvumul_noovfl": "UMUL_NOOVF",
}
_SWAPPED = {"bvugt": "ULT", "bvuge": "ULE", "bvsgt": "SLT", "bvsge": "SLE"}


class Unsupported(Exception):
    """The query uses a construct the engine does not evaluate (-> z3)."""


def limbs(w: int) -> int:
    return (w + 31) // 32


def int_to_limbs(v: int, w: int) -> List[int]:
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(limbs(w))]


def limbs_to_int(ws: Sequence[int]) -> int:
    v = 0
    for i, x in enumerate(ws):
        v |= (int(x) & 0xFFFFFFFF) << (32 * i)
    return v


class Coord:
    __slots__ = ("index", "width", "kind", "node", "table", "name", "term")

    def __init__(self, index, width, kind, node, table, name, term):
        self.index, self.width, self.kind, self.node = index, width, kind, node
        self.table, self.name, self.term = table, name, term

    def __repr__(self):
        return f"Coord({self.index}, {self.name}, w={self.width}, kind={self.kind})"


class Table:
    __slots__ = ("index", "kind", "name", "key_width", "val_width")

    def __init__(self, index, kind, name, kw, vw):
        self.index, self.kind, self.name, self.key_width, self.val_width = index, kind, name, kw, vw


class Program:
    """A flattened query: the v1 bytes plus the host-side metadata needed to
    build inputs and read models back."""

    def __init__(self):
        self.nodes: List[List[int]] = []
        self.node_width: List[int] = []
        self.roots: List[int] = []
        self.coords: List[Coord] = []
        self.tables: List[Table] = []
        self.consts: List[int] = []
        self.watch: List[int] = []
        self.term_node: Dict[int, int] = {}     # term id -> node index
        self.node_term: List[Optional[T.Term]] = []
        self.sites: List[Coord] = []            # coords of array/UF sites, in SSA order
        self.site_key_node: Dict[int, int] = {}  # coord index -> node of the key
        self.site_val_node: Dict[int, int] = {}  # coord index -> node of the site value
        self.const_values: List[tuple] = []      # (value, width) of every literal, for dictionaries
        self.aux_slice: Dict[int, tuple] = {}     # site coord -> (AUX coord, bit offset) of its lazy default
        self._blob: Optional[bytes] = None

    # -- properties --------------------------------------------------
    @property
    def coord_words(self) -> int:
        return sum(limbs(c.width) for c in self.coords)

    def coord_row_offsets(self) -> List[int]:
        out, r = [], 0
        for c in self.coords:
            out.append(r)
            r += limbs(c.width)
        return out

    def watch_width(self, entry: int) -> int:
        """Width of a watch entry: a node, or 0x80000000 | coord for a site's base value."""
        return self.coords[entry & 0x7FFFFFFF].width if entry & 0x80000000 else self.node_width[entry]

    @property
    def watch_words(self) -> int:
        return sum(limbs(self.watch_width(n)) for n in self.watch)

    def watch_row_offsets(self) -> List[int]:
        out, r = [], 0
        for n in self.watch:
            out.append(r)
            r += limbs(self.watch_width(n))
        return out

    def scalar_coords(self):
        return [c for c in self.coords if c.kind == COORD_SCALAR]

    def set_watch(self, nodes: Iterable[int]):
        self.watch = list(nodes)
        self._blob = None

    def watch_terms(self, terms: Iterable[T.Term]):
        self.set_watch([self.term_node[t.id] for t in terms])

    def to_bytes(self) -> bytes:
        if self._blob is not None:
            return self._blob
        hdr = [MG_MAGIC, MG_VERSION, len(self.nodes), len(self.roots), len(self.coords),
               len(self.tables), len(self.consts), len(self.watch)] + [0] * 8
        words = list(hdr)
        for n in self.nodes:
            words.extend(n)
        words.extend(self.roots)
        for c in self.coords:
            words.extend([c.width, c.kind, c.node, c.table if c.table is not None else MG_NONE])
        for t in self.tables:
            words.extend([t.kind, t.key_width, t.val_width, 0])
        words.extend(self.watch)
        words.extend(self.consts)
        self._blob = struct.pack(f"<{len(words)}I", *words)
        return self._blob


def _base_of(arr: T.Term) -> T.Term:
    while arr.op == "store":
        arr = arr.args[0]
    return arr


def calldata_window(name: str, dom: int, rng: int, index: int):
    """The AUX word a calldata byte belongs to (``aux_words`` flattening), or None.

    LASER's calldata is the array ``<tx>_calldata`` (256 -> 8, ``calldata.py:215-216``)
    and ABI data is a 4-byte selector followed by 32-byte words read with
    CALLDATALOAD (``instructions.py:775-789``, ``calldata.py:47-54``): byte k belongs
    to the selector window [0, 4) or to the word [4 + 32m, 36 + 32m).  Returns
    ``(start, length)``.  The window depends on the index alone, so prefix-incremental
    flattening stays byte-identical."""
    if not name.endswith("_calldata") or dom != 256 or rng != 8 or index >= 1 << 32:
        return None
    if index < 4:
        return 0, 4
    return 4 + 32 * ((index - 4) // 32), 32


def _extend(st: "_FlatState", terms: Sequence[T.Term], lazy_inverse: bool) -> None:
    """Flatten the not-yet-flattened subterms of ``terms`` into ``st.P``."""
    P = st.P
    scalar_coord, table_of, fwd_arg = st.scalar_coord, st.table_of, st.fwd_arg

    nodes, node_width, node_term, term_node = P.nodes, P.node_width, P.node_term, P.term_node

    def new_node(op, width, a=MG_NONE, b=MG_NONE, c=MG_NONE, p0=0, p1=0, p2=0, term=None):
        if width > MG_MAX_WIDTH:
            raise Unsupported(f"width {width} > {MG_MAX_WIDTH}")
        nodes.append([OPS[op], width, a, b, c, p0, p1, p2])
        node_width.append(width)
        node_term.append(term)
        return len(nodes) - 1

    def const_node(v: int, w: int, term=None):
        off = len(P.consts)
        P.consts.extend(int_to_limbs(v, w))
        P.const_values.append((v, w))
        return new_node("CONST", w, p0=off, term=term)

    def table(kind, name, kw, vw):
        # keyed by name alone: the model (Model.arrays / funcs) is keyed by name, so one
        # name at two sorts would silently merge two tables there
        key = (kind, name)
        t = table_of.get(key)
        if t is None:
            t = len(P.tables)
            P.tables.append(Table(t, kind, name, kw, vw))
            table_of[key] = t
        elif (P.tables[t].key_width, P.tables[t].val_width) != (kw, vw):
            raise Unsupported(f"symbol {name} used with two sorts")
        return t

    def new_coord(width, kind, node, tab, name, term):
        c = Coord(len(P.coords), width, kind, node, tab, name, term)
        P.coords.append(c)
        return c

    order = T.postorder(terms, skip=P.term_node) if P.term_node else T.postorder(terms)
    for t in order:
        if lazy_inverse and t.op == "app":
            # forward UF apps, for lazy inverse defaults; the argument of an inverse
            # app is visited before it (children first), so one pass suffices
            fwd_arg[t.id] = t.args[0].id
    def nid(x):
        return term_node[x.id]

    for t in order:
        n = None
        op = t.op
        if op in ("bvconst", "boolconst"):
            n = const_node(T.const_value(t), t.width, term=t)
        elif op in ("bvvar", "boolvar"):
            name = t.params[0]
            # keyed by name alone (Model.scalars is): a second sort of the same name is
            # a different z3 constant that this model layout cannot represent
            key = name
            if key in scalar_coord:
                raise Unsupported(f"symbol {name} used with two sorts")
            ci = len(P.coords)
            n = new_node("VAR", t.width, p0=ci, term=t)
            new_coord(t.width, COORD_SCALAR, n, None, name, t)
            scalar_coord[key] = ci
        elif op in _BIN:
            n = new_node(_BIN[op], t.width, nid(t.args[0]), nid(t.args[1]), term=t)
        elif op in _SWAPPED:
            n = new_node(_SWAPPED[op], 1, nid(t.args[1]), nid(t.args[0]), term=t)
        elif op == "bvnot":
            n = new_node("NOT", t.width, nid(t.args[0]), term=t)
        elif op == "bvneg":
            n = new_node("NEG", t.width, nid(t.args[0]), term=t)
        elif op == "concat":
            n = new_node("CONCAT", t.width, nid(t.args[0]), nid(t.args[1]), term=t)
        elif op == "extract":
            n = new_node("EXTRACT", t.width, nid(t.args[0]), p0=t.params[1], term=t)
        elif op == "zero_extend":
            n = new_node("ZEXT", t.width, nid(t.args[0]), term=t)
        elif op == "sign_extend":
            n = new_node("SEXT", t.width, nid(t.args[0]), term=t)
        elif op == "ite":
            if t.is_array:
                raise Unsupported("ite over arrays")
            n = new_node("ITE", t.width, nid(t.args[0]), nid(t.args[1]), nid(t.args[2]), term=t)
        elif op == "eq":
            if t.args[0].is_array:
                raise Unsupported("array equality")
            n = new_node("EQ", 1, nid(t.args[0]), nid(t.args[1]), term=t)
        elif op in ("and", "or"):
            acc = nid(t.args[0])
            for x in t.args[1:]:
                acc = new_node("AND" if op == "and" else "OR", 1, acc, nid(x))
            n = acc
            P.node_term[n] = t
        elif op == "not":
            n = new_node("NOT", 1, nid(t.args[0]), term=t)
        elif op == "xor":
            n = new_node("XOR", 1, nid(t.args[0]), nid(t.args[1]), term=t)
        elif op == "array_var":
            _, d, r = t.sort
            tab = table(TABLE_ARRAY, t.params[0], d, r)
            n = new_node("ARR_VAR", 0, p0=tab, term=t)
        elif op == "const_array":
            n = new_node("ARR_K", 0, nid(t.args[0]), term=t)
        elif op == "store":
            n = new_node("ARR_STORE", 0, nid(t.args[0]), nid(t.args[1]), nid(t.args[2]), term=t)
        elif op == "select":
            base = _base_of(t.args[0])
            if base.op == "array_var":
                tab = P.nodes[nid(base)][5]
                lazy = MG_NONE
                idx = t.args[1]
                win = None
                if st.aux_words and base is t.args[0] and idx.op == "bvconst":
                    win = calldata_window(base.params[0], base.sort[1], base.sort[2], idx.params[0])
                if win is not None:
                    # the byte is a slice of a generator-only AUX word (one 256-bit draw per
                    # ABI word instead of 32 byte draws); the site's table entry is still
                    # read back as the model
                    key = (base.params[0], win[0])
                    if key not in st.aux_of:
                        wbits = 8 * win[1]
                        an = new_node("VAR", wbits, p0=len(P.coords))
                        ac = new_coord(wbits, COORD_AUX, an, None, f"{base.params[0]}@{win[0]}", None)
                        st.aux_of[key] = (ac.index, an)
                    ac_i, an = st.aux_of[key]
                    b = 8 * (win[0] + win[1] - 1 - idx.params[0])
                    lazy = new_node("EXTRACT", 8, an, p0=b)
                    P.aux_slice[len(P.coords)] = (ac_i, b)
                n = new_node("SELECT", t.width, nid(t.args[0]), nid(t.args[1]), p0=len(P.coords), p1=lazy,
                             term=t)
                c = new_coord(t.width, COORD_ARRAY_SITE, n, tab, base.params[0], t)
                P.sites.append(c)
                P.site_key_node[c.index] = nid(t.args[1])
                P.site_val_node[c.index] = n
            elif base.op == "const_array":
                n = new_node("SELECT", t.width, nid(t.args[0]), nid(t.args[1]), p0=MG_NONE, p1=MG_NONE, term=t)
            else:
                raise Unsupported(f"select over {base.op}")
        elif op == "app":
            fname, dom, rng = t.params
            tab = table(TABLE_UF, fname, dom, rng)
            arg = t.args[0]
            lazy = MG_NONE
            if lazy_inverse and arg.id in fwd_arg and fname.endswith("-1"):
                src = fwd_arg[arg.id]
                if src in P.term_node and P.node_width[P.term_node[src]] == rng:
                    lazy = P.term_node[src]
            n = new_node("UFAPP", rng, nid(arg), p0=tab, p1=len(P.coords), p2=lazy, term=t)
            c = new_coord(rng, COORD_UF_SITE, n, tab, fname, t)
            P.sites.append(c)
            P.site_key_node[c.index] = nid(arg)
            P.site_val_node[c.index] = n
        elif op == "keccak256":
            if t.args:
                w = t.args[0].width
                n = new_node("KECCAK", 256, nid(t.args[0]), p0=w // 8, term=t)
            else:
                n = new_node("KECCAK", 256, MG_NONE, p0=0, term=t)
        else:
            raise Unsupported(f"operator {op}")
        P.term_node[t.id] = n

    P._blob = None


def flatten(roots: Sequence[T.Term], lazy_inverse: bool = True, extra: Sequence[T.Term] = (),
            aux_words: bool = False) -> Program:
    """Flatten Bool roots (terms) into a :class:`Program`.  ``extra`` terms are
    flattened too (so they can be watched) without becoming constraints.

    ``aux_words`` (search mode): literal-index calldata bytes take their default from
    a generator-only AUX word (:func:`calldata_window`) instead of a coordinate of
    their own, so explicit-coordinate evaluation (``mg_eval``) leaves it off."""
    roots = list(roots)
    for r in roots:
        if not r.is_bool:
            raise TypeError("constraint roots must be Bool terms")
    st = _FlatState(aux_words)
    _extend(st, list(roots) + list(extra), lazy_inverse)
    st.P.roots = [st.P.term_node[r.id] for r in roots]
    return st.P


class _FlatState:
    """A Program under construction plus the flattener's lookup tables."""

    def __init__(self, aux_words: bool = False):
        self.P = Program()
        self.scalar_coord: Dict[str, int] = {}
        self.table_of: Dict[tuple, int] = {}
        self.fwd_arg: Dict[int, int] = {}   # term id of f(x) app -> term id of x
        self.aux_words = aux_words
        self.aux_of: Dict[tuple, tuple] = {}  # (calldata array, window start) -> (AUX coord, VAR node)

    def copy(self) -> "_FlatState":
        c = _FlatState(self.aux_words)
        P, Q = self.P, c.P
        Q.nodes = [list(n) for n in P.nodes]
        Q.node_width = list(P.node_width)
        Q.roots = list(P.roots)
        Q.coords = list(P.coords)
        Q.tables = list(P.tables)
        Q.consts = list(P.consts)
        Q.term_node = dict(P.term_node)
        Q.node_term = list(P.node_term)
        Q.sites = list(P.sites)
        Q.site_key_node = dict(P.site_key_node)
        Q.site_val_node = dict(P.site_val_node)
        Q.const_values = list(P.const_values)
        Q.aux_slice = dict(P.aux_slice)
        c.aux_of = dict(self.aux_of)
        c.scalar_coord = dict(self.scalar_coord)
        c.table_of = dict(self.table_of)
        c.fwd_arg = dict(self.fwd_arg)
        return c


class FlattenCache:
    """Prefix-incremental flattening.

    LASER's states share constraint prefixes: ``Constraints.__copy__`` /
    ``WorldState.__copy__`` (``constraints.py:61-98``, ``world_state.py:58-74``)
    hand each successor its parent's list, and ``svm.py:252-257`` then appends
    one JUMPI condition.  The flattened state after every root prefix is kept
    (keyed by the root term ids, LRU); a query extends the longest cached prefix
    with its remaining roots only.  Terms are hash-consed, so the program built
    this way is byte-identical to :func:`flatten` of the whole tuple
    (``tests/test_host_boundary.py``)."""

    def __init__(self, capacity: int = 4096, lazy_inverse: bool = True, aux_words: bool = False):
        from collections import OrderedDict

        self.capacity, self.lazy_inverse, self.aux_words = capacity, lazy_inverse, aux_words
        self._lru: "OrderedDict[tuple, _FlatState]" = OrderedDict()
        self.hits = self.misses = 0

    def flatten(self, roots: Sequence[T.Term]) -> Program:
        roots = list(roots)
        for r in roots:
            if not r.is_bool:
                raise TypeError("constraint roots must be Bool terms")
        ids = tuple(r.id for r in roots)
        k = len(ids)
        while k > 0 and ids[:k] not in self._lru:
            k -= 1
        if k:
            self.hits += 1
            self._lru.move_to_end(ids[:k])
            st = self._lru[ids[:k]].copy()
        else:
            self.misses += 1
            st = _FlatState(self.aux_words)
        if k == len(ids):
            return st.P
        _extend(st, roots[k:], self.lazy_inverse)
        st.P.roots.extend(st.P.term_node[r.id] for r in roots[k:])
        self._put(ids, st.copy())  # a query's successors extend its own tuple (svm.py:252-257)
        return st.P

    def _put(self, key, st):
        self._lru[key] = st
        self._lru.move_to_end(key)
        while len(self._lru) > self.capacity:
            self._lru.popitem(last=False)


# ---------------------------------------------------------------------------
# inputs and models
# ---------------------------------------------------------------------------

def soa_from_assignments(P: Program, assignments: Sequence[Sequence[int]]):
    """Build the ``[coord row][candidate]`` uint32 SoA for :func:`mg_eval`.

    ``assignments[i][c]`` is the integer value of coordinate ``c`` for candidate ``i``.
    Returns a numpy array of shape (coord_words, n)."""
    import numpy as np

    n = len(assignments)
    rows = P.coord_words
    out = np.zeros((max(rows, 1), n), dtype=np.uint32)
    offs = P.coord_row_offsets()
    for c in P.coords:
        L = limbs(c.width)
        mask = (1 << c.width) - 1
        col = [int(a[c.index]) & mask for a in assignments]
        for j in range(L):
            out[offs[c.index] + j, :] = [(v >> (32 * j)) & 0xFFFFFFFF for v in col]
    return out


def model_from_sites(P: Program, scalar_vals: Dict[int, int], site_keys: Dict[int, int],
                     site_vals: Dict[int, int]):
    """Turn one evaluated candidate into a finite model (first site wins per key).

    Returns ``(scalars, arrays, funcs)`` with ``arrays``/``funcs`` as
    ``name -> ({key: value}, else=0)``."""
    scalars = {c.name: scalar_vals[c.index] for c in P.scalar_coords() if c.index in scalar_vals}
    arrays: Dict[str, tuple] = {}
    funcs: Dict[str, tuple] = {}
    for c in P.sites:
        if c.index not in site_keys:
            continue
        tgt = arrays if c.kind == COORD_ARRAY_SITE else funcs
        table, _ = tgt.setdefault(c.name, ({}, 0))
        k = site_keys[c.index]
        if k not in table:
            table[k] = site_vals[c.index]
    return scalars, arrays, funcs
