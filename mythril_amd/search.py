"""Candidate generation, GPU search and model materialisation.

This is the engine's answer to ``Optimize.check()`` for SAT instances
(``mythril/support/model.py:44``): sweep candidate indices on the GPU until one
satisfies every constraint, then read the winning candidate back as a finite
model (``Solver.model()``, ``laser/smt/solver/solver.py:59-64``).

Generator heuristics (per coordinate, all on device, pure functions of
``(seed, index, coordinate)`` so the first hit is the same on any GPU count):

* scalars: a MIXED draw over a dictionary of the query's own literals of that
  width (plus 0, 1, 2^w-1, the three LASER actor addresses of
  ``transaction/symbolic.py:22-33``), +/-1/2 around them, copies of another
  coordinate of the same width (equalities between symbols are common),
  small values (calldatasize, loop counters), and uniform bits;
* keccak UF sites: multiples of 64 inside the interval the side condition
  pins (``keccak_function_manager.py:121-149``), read from the query's own
  constants (never recomputed);
* inverse-UF sites: lazily equal to the forward argument (set in ``ssa.py``).
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import ssa
from .smt import terms as T

GEN_MAGIC = 0x334E4547  # "GEN3" (include/mythgpu.h)
GEN_UNIFORM, GEN_RANGE, GEN_DICT, GEN_MIXED, GEN_ALIGNED, GEN_FIXED, GEN_LAZY = range(7)
NONE = ssa.MG_NONE

ACTORS = [
    0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,  # CREATOR  (transaction/symbolic.py:22-33)
    0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,  # ATTACKER
    0xAAAAAAAABBBBBBBBCCCCCCCCDDDDDDDDEEEEEEEE,  # SOMEGUY
]

P16 = 65536
MAX_COPY_DEPTH = 16  # <= MG_GEN_MAX_COPY_DEPTH (include/mythgpu.h)

# prefix-incremental flattening shared by every search (LASER's sibling queries share prefixes)
FLATTEN_CACHE = ssa.FlattenCache(aux_words=True)

# A generator bound, not a fact of the query: LASER's ``<tx>_calldatasize``
# (calldata.py:215-216) is a 256-bit symbol, but a transaction's calldata is paid
# per byte and bounded by the block gas limit, so no realisable model has 2^32 bytes
# of it.  Sizes are drawn inside [0, 2^32) (then the query's own bounds).
CALLDATASIZE_MAX = (1 << 32) - 1


class GenBuilder:
    """Assemble a generator blob (``include/mythgpu.h`` MG_GEN_MAGIC layout)."""

    def __init__(self, P: ssa.Program):
        self.P = P
        self.specs: List[List[int]] = [[GEN_UNIFORM, 0, 0, 0, 0, 0, 0, 0] for _ in P.coords]
        self.consts: List[int] = []
        self._pool: Dict[tuple, int] = {}  # (width, values) -> offset: coordinates share dictionaries

    def _push(self, values: Sequence[int], w: int) -> int:
        key = (w, tuple(values))
        off = self._pool.get(key)
        if off is not None:
            return off
        off = len(self.consts)
        L = ssa.limbs(w)
        m = (1 << w) - 1
        raw = b"".join((int(v) & m).to_bytes(4 * L, "little") for v in values)
        self.consts.extend(np.frombuffer(raw, dtype="<u4").tolist())
        self._pool[key] = off
        return off

    def uniform(self, c: int):
        self.specs[c] = [GEN_UNIFORM, 0, 0, 0, 0, 0, 0, 0]

    def fixed(self, c: int, v: int):
        w = self.P.coords[c].width
        self.specs[c] = [GEN_FIXED, self._push([v], w), 0, 0, 0, 0, 0, 0]

    def range(self, c: int, lo: int, span: int):
        w = self.P.coords[c].width
        self.specs[c] = [GEN_RANGE, self._push([lo], w), span & 0xFFFFFFFF, 0, 0, 0, 0, 0]

    def dict(self, c: int, values: Sequence[int]):
        w = self.P.coords[c].width
        self.specs[c] = [GEN_DICT, self._push(values, w), len(values), 0, 0, 0, 0, 0]

    def aligned(self, c: int, lo: int, log2_align: int, count: int):
        w = self.P.coords[c].width
        self.specs[c] = [GEN_ALIGNED, self._push([lo], w), log2_align, min(count, 1 << 32) & 0xFFFFFFFF,
                         0, 0, 0, 0]

    def lazy(self, c: int):
        self.specs[c] = [GEN_LAZY, 0, 0, 0, 0, 0, 0, 0]

    def mixed(self, c: int, values: Sequence[int], p_dict: float, copy_from: Optional[int] = None,
              p_copy: float = 0.0, p_delta: float = 0.0, small_bits: int = 0, p_small: float = 0.0,
              clamp: Optional[tuple] = None):
        """MIXED (GEN3): one alternative per aligned group of 64 candidates — COPY of an
        earlier coordinate's final value, DICT, SMALL or UNIFORM — plus a per-lane +/-1/2
        delta on COPY/DICT, then an optional clamp into ``[lo, lo + span)``."""
        w = self.P.coords[c].width
        values = list(values)
        off = self._push(values, w) if values else 0
        pc = int(p_copy * P16) if copy_from is not None else 0
        pd = int(p_dict * P16) if values else 0
        rec = 0
        if clamp is not None:
            lo, span = clamp
            rec = len(self.consts) + 1
            self.consts.extend(ssa.int_to_limbs(lo % (1 << w), w))
            self.consts.append(span & 0xFFFFFFFF)
        self.specs[c] = [
            GEN_MIXED, off, len(values), (pc & 0xFFFF) | ((pd & 0xFFFF) << 16),
            NONE if copy_from is None else copy_from,
            (int(p_small * P16) & 0xFFFF) | ((small_bits & 0xFFFF) << 16), int(p_delta * P16) & 0xFFFF, rec,
        ]

    def fix(self, c: int, mask: int, value: int):
        """Fixed bits applied after generation: v = (v & ~mask) | value (call last)."""
        w = self.P.coords[c].width
        mask &= (1 << w) - 1
        if not mask:
            return
        off = len(self.consts)
        self.consts.extend(ssa.int_to_limbs(mask, w))
        self.consts.extend(ssa.int_to_limbs(value & mask, w))
        self.specs[c][0] = (self.specs[c][0] & 0xFF) | ((off + 1) << 8)

    def blob(self) -> np.ndarray:
        head = np.array([GEN_MAGIC, len(self.specs), len(self.consts), 0], dtype=np.uint32)
        specs = np.array(self.specs, dtype=np.int64).astype(np.uint32).reshape(-1)
        return np.concatenate([head, specs, np.array(self.consts, dtype=np.uint32)])


def _interval_bounds(P: ssa.Program):
    """For each UF-site coordinate, the [lo, hi) literal bounds the query puts on
    the application (ULE(lo, f(x)) / ULT(f(x), hi), keccak_function_manager.py:138-143)."""
    out: Dict[int, list] = {}
    site_of_node = {P.site_val_node[c.index]: c.index for c in P.sites}
    for n, node in enumerate(P.nodes):
        op = node[0]
        if op not in (ssa.OPS["ULT"], ssa.OPS["ULE"]):
            continue
        a, b = node[2], node[3]
        ta, tb = P.node_term[a], P.node_term[b]
        if b in site_of_node and ta is not None and ta.op == "bvconst":
            lo = ta.params[0]
            out.setdefault(site_of_node[b], [None, None])[0] = lo if op == ssa.OPS["ULE"] else lo + 1
        if a in site_of_node and tb is not None and tb.op == "bvconst":
            hi = tb.params[0]
            out.setdefault(site_of_node[a], [None, None])[1] = hi if op == ssa.OPS["ULT"] else hi + 1
    return out


def default_generator(P: ssa.Program, extra_dict: Sequence[int] = (), roots: Optional[Sequence[T.Term]] = None
                      ) -> GenBuilder:
    """Per-coordinate generator specs.  With ``roots`` the propagation pass
    (``propagate.py``) first shapes each coordinate's domain."""
    from .propagate import propagate

    doms = propagate(P, roots) if roots is not None else {}
    g = GenBuilder(P)
    by_width: Dict[int, set] = {}
    for v, w in P.const_values:
        by_width.setdefault(w, set()).add(v)
    bounds = _interval_bounds(P)
    last_of_width: Dict[int, int] = {}
    depth: Dict[int, int] = {}  # COPY chain length per coordinate (MG_GEN_MAX_COPY_DEPTH bounds it)
    for c in P.coords:
        w = c.width
        mask = (1 << w) - 1
        if (c.kind == ssa.COORD_UF_SITE and P.nodes[c.node][7] != NONE) or \
                (c.kind == ssa.COORD_ARRAY_SITE and P.nodes[c.node][6] != NONE):
            g.lazy(c.index)  # the program supplies the default (inverse UF argument, AUX word byte)
            continue
        dom = doms.get(c.index)
        if c.kind == ssa.COORD_SCALAR and c.name.endswith("_calldatasize") and w > 32:
            from .propagate import Domain

            dom = dom or Domain(w)
            if not dom.restrict([(0, CALLDATASIZE_MAX)]):
                dom = None
        if dom is not None and _apply_domain(g, P, c.index, dom):
            last_of_width[w] = c.index
            continue
        if dom is None and c.kind == ssa.COORD_UF_SITE and c.index in bounds and None not in bounds[c.index]:
            lo, hi = bounds[c.index]
            lo = (lo + 63) // 64 * 64
            if hi > lo:
                g.aligned(c.index, lo, 6, max(1, (hi - lo) // 64))
                continue
        if w == 1:
            g.uniform(c.index)
            last_of_width[w] = c.index
            continue
        vals = set(by_width.get(w, ())) | {0, 1, mask}
        for a in list(ACTORS) + list(extra_dict):
            vals.add(a & mask)
        small_bits, p_small = min(w, 8), 0.20
        clamp = None
        if dom is not None:
            if dom.intervals:
                for a_, b_ in dom.intervals[:4]:
                    vals |= {a_, (a_ + 1) & mask, b_, (b_ - 1) & mask}
                a_, b_ = dom.intervals[0][0], dom.intervals[-1][1]
                if len(dom.intervals) == 1 and b_ - a_ < (1 << 32):
                    clamp = (a_, (b_ - a_ + 1) & 0xFFFFFFFF)  # span 2^32 is encoded as 0
            vals = {v for v in vals if dom.admissible(v)} or vals
        vals = sorted(vals)[:4096]
        copy = last_of_width.get(w) if w >= 32 else None
        if copy is not None and depth.get(copy, 0) >= MAX_COPY_DEPTH:
            copy = None  # start a new chain (the interpreter walks chains per candidate)
        depth[c.index] = depth.get(copy, 0) + 1 if copy is not None else 0
        g.mixed(c.index, vals, p_dict=0.45, copy_from=copy, p_copy=0.10 if copy is not None else 0.0,
                p_delta=0.25 if w > 8 else 0.0, small_bits=small_bits, p_small=p_small, clamp=clamp)
        if dom is not None and dom.fmask:
            g.fix(c.index, dom.fmask, dom.fval)
        last_of_width[w] = c.index
    return g


def _apply_domain(g: GenBuilder, P: ssa.Program, c: int, dom) -> bool:
    """Give coordinate c a spec drawn from its propagated domain when the domain is
    narrow enough to enumerate; False leaves it to the broad default draw."""
    w = P.coords[c].width
    full = (1 << w) - 1
    if dom.choices:
        ok = [v for v in dom.choices if dom.admissible(v)]
        if ok:
            g.dict(c, ok)
            return True
    if dom.fmask == full:
        g.fixed(c, dom.fval)
        return True
    if dom.intervals:
        a, b = dom.intervals[0]
        # low zero bits fixed (keccak outputs: URem(f(x), 64) == 0) -> aligned sweep
        k = 0
        while k < w and (dom.fmask >> k) & 1 and not (dom.fval >> k) & 1:
            k += 1
        if k:
            lo = (a + (1 << k) - 1) >> k << k
            if lo <= b:
                g.aligned(c, lo, k, min(((b - lo) >> k) + 1, 1 << 32) % (1 << 32))
                rest = dom.fmask & ~((1 << k) - 1)
                if rest:
                    g.fix(c, rest, dom.fval)
                return True
        span = sum(y - x + 1 for x, y in dom.intervals)
        if span <= (1 << 16) and len(dom.intervals) == 1:
            g.range(c, a, span)
            if dom.fmask:
                g.fix(c, dom.fmask, dom.fval)
            return True
    return False


class SearchResult:
    def __init__(self, index, hits, scanned, seconds, model=None):
        self.index, self.hits, self.scanned, self.seconds, self.model = index, hits, scanned, seconds, model
        self.engine = "interp"
        self.buckets = 1
        self.timing = {}


def _const_node_value(P: ssa.Program, node: int) -> Optional[int]:
    """The value of a literal node (host-known), else None."""
    t = P.node_term[node] if node < len(P.node_term) else None
    return t.params[0] if t is not None and t.op == "bvconst" else None


def _model_layout(P: ssa.Program):
    """The model read-back layout (built once per Program, ``P._model_layout``).

    A model is the scalar coordinates plus one (key, value) table entry per array/UF site
    (``ssa.model_from_sites``).  What the host already knows is not read back from the GPU:
    a site key that is a literal (``Select(<tx>_calldata, k)`` at a literal index, a literal
    storage slot), and the value of a calldata site whose default is a byte of an AUX word
    (``ssa.calldata_window``: read the word once, slice the bytes on the host).  So the watch
    list is: scalar VAR nodes, AUX word VAR nodes, then per site its key node (unless literal)
    and its base value (``0x80000000 | coord``, unless AUX-sliced).

    Returns (entries, widths, plan); plan = (scalars [(entry position, name)], aux {coord:
    position}, sites [(name, is_array, key position or None, literal key, base position or
    None, (aux coord, bit offset, width) or None)])."""
    lay = getattr(P, "_model_layout", None)
    if lay is not None:
        return lay
    entries, widths = [], []

    def add(e, w):
        entries.append(e)
        widths.append(w)
        return len(entries) - 1

    scal = [(add(c.node, c.width), c.name) for c in P.scalar_coords()]
    aux_used = {a for a, _ in P.aux_slice.values()}
    aux = {c.index: add(c.node, c.width) for c in P.coords if c.kind == ssa.COORD_AUX and c.index in aux_used}
    sites = []
    for c in P.sites:
        k = P.site_key_node[c.index]
        lit = _const_node_value(P, k)
        kpos = None if lit is not None else add(k, P.node_width[k])
        sl = P.aux_slice.get(c.index)
        if sl is not None:
            bpos, slc = None, (sl[0], sl[1], c.width)
        else:
            bpos, slc = add(0x80000000 | c.index, c.width), None
        sites.append((c.name, c.kind == ssa.COORD_ARRAY_SITE, kpos, lit, bpos, slc))
    lay = (entries, widths, (scal, aux, sites))
    P._model_layout = lay
    return lay


def model_watch(P: ssa.Program):
    """Watch entries that read a whole model back (``_model_layout``): (entries, widths)."""
    entries, widths, _ = _model_layout(P)
    return entries, widths


def decode_model(P: ssa.Program, vals: Sequence[int]):
    """(scalars, arrays, funcs) from the values of P's model watch entries, in order: the
    finite z3 model of one candidate (first site wins per key, as ``ssa.model_from_sites``)."""
    _, _, (scal, aux, sites) = _model_layout(P)
    scalars = {name: vals[i] for i, name in scal}
    arrays: dict = {}
    funcs: dict = {}
    for name, is_array, kpos, lit, bpos, slc in sites:
        table = (arrays if is_array else funcs).setdefault(name, ({}, 0))[0]
        k = lit if kpos is None else vals[kpos]
        if k in table:
            continue
        if bpos is not None:
            table[k] = vals[bpos]
        else:
            a, off, w = slc
            table[k] = (vals[aux[a]] >> off) & ((1 << w) - 1)
    return scalars, arrays, funcs


def read_rows(watch: np.ndarray, widths: Sequence[int], col: int) -> List[int]:
    out, r = [], 0
    for w in widths:
        L = ssa.limbs(w)
        out.append(ssa.limbs_to_int(watch[r:r + L, col]))
        r += L
    return out


def materialize(engine, P: ssa.Program, gen_blob: np.ndarray, seed: int, index: int):
    """Re-run candidate ``index`` with the model watch list; returns (verdict, scalars, arrays, funcs)."""
    entries, widths = model_watch(P)
    prev = P.watch
    P.set_watch(entries)
    prog = engine.load(P.to_bytes())
    try:
        gen = engine.load_gen(prog, gen_blob)
        try:
            ver, watch = engine.eval_generated(prog, gen, seed, index, 1, watch_words=sum(ssa.limbs(w) for w in widths))
        finally:
            engine.free_gen(gen)
    finally:
        engine.free(prog)
        P.set_watch(prev)
    vals = read_rows(watch, widths, 0) if watch is not None else []
    scalars, arrays, funcs = decode_model(P, vals)
    return int(ver[0]), scalars, arrays, funcs


def prepare(roots: Sequence[T.Term], gen: Optional[GenBuilder] = None):
    """The program and generator blob a search runs: prefix-incremental flattening with
    AUX calldata words (``FLATTEN_CACHE``), the model watch list (``model_watch``: what
    ``mg_search``'s ``assign_out`` returns for the winning candidate) and the
    propagation-shaped generator.

    The whole result is a pure function of the (hash-consed) roots, and LASER re-asks the
    same constraint set (``is_possible``, then the detection modules): a repeat returns the
    SAME Program object (its serialised bytes and model read-back plan already built), so
    callers must not mutate it."""
    if gen is not None:
        P = FLATTEN_CACHE.flatten(roots)
        P.set_watch(model_watch(P)[0])
        return P, gen.blob()
    key = tuple(t.id for t in roots)
    hit = _GEN_CACHE.get(key)
    if hit is not None:
        _GEN_CACHE[key] = _GEN_CACHE.pop(key)  # most recent last
        return hit
    P = FLATTEN_CACHE.flatten(roots)
    P.set_watch(model_watch(P)[0])
    blob = default_generator(P, roots=roots).blob()
    _GEN_CACHE[key] = (P, blob)
    if len(_GEN_CACHE) > _GEN_CACHE_MAX:
        _GEN_CACHE.pop(next(iter(_GEN_CACHE)))
    return P, blob


_GEN_CACHE: "dict" = {}
_GEN_CACHE_MAX = 512


def _model_plan(P: ssa.Program):
    """Byte slices of P's model watch rows in an ``assign_out`` buffer (built once)."""
    plan = getattr(P, "_model_plan", None)
    if plan is None:
        _, widths = model_watch(P)
        plan, r = [], 0
        for w in widths:
            L = ssa.limbs(w)
            plan.append((4 * r, 4 * (r + L)))
            r += L
        P._model_plan = plan
    return plan


def model_from_assignment(P: ssa.Program, assign: np.ndarray):
    """(scalars, arrays, funcs) from the watch rows ``mg_search`` wrote for a hit."""
    raw = np.ascontiguousarray(assign, dtype="<u4").tobytes()
    fb = int.from_bytes
    return decode_model(P, [fb(raw[a:b], "little") for a, b in _model_plan(P)])


# expected latency of one query-kernel compile (submit -> loadable module), seconds: an
# exponential average of the compiles this process measured (cold value from the bench:
# ~0.2 s on the MI355X box's host through hipRTC, less through comgr)
JIT_COMPILE_S = [0.15]
# the same for the first tier (assembly emitted by the engine, jit_asm.cpp): emission + assembler
# + link, a few ms
JIT_ASM_COMPILE_S = [0.01]
# MYTHGPU_JIT_ASM=0: no first tier (the interpreter runs until the O3 kernel is ready)
JIT_ASM = os.environ.get("MYTHGPU_JIT_ASM", "1") != "0"
# while a compile is pending, interpreter launches are cut to about this long so the search
# switches to the compiled kernel soon after it is ready; in the first few ms after the submit they
# are cut to JIT_FIRST_POLL_S, so a kernel the engine already holds (same source: LASER re-asks
# constraint sets) is picked up at once instead of after a full 10 ms interpreter launch
JIT_POLL_S = 0.010
JIT_FIRST_POLL_S = 0.001
# the tier race (first tier against the O3 kernel on the same query): the first tier is kept only when
# it is faster by more than this fraction
RACE_TIE = 0.03
# kernel that produced the last search's result ("interp" / "jit") and that result, for
# stream statistics (tools/stream_bench.py)
LAST_ENGINE = None
LAST_RESULT = None


def search(engine, roots: Sequence[T.Term], seed: int = 0x6D797468, chunk: int = 1 << 12,
           max_candidates: int = 1 << 26, timeout_s: float = 10.0, gen: Optional[GenBuilder] = None,
           want_model: bool = True, jit: str = "auto", jit_cost_s: Optional[float] = None,
           cancel=None, max_launch_s: Optional[float] = None) -> SearchResult:
    """Find the lowest-index satisfying candidate (or give up: None).

    ``jit``: "never" keeps the generic interpreter (``k_run``, no compile latency);
    "always" compiles the query-specialised kernel first; "auto" starts on the
    interpreter and, when the first launch has no hit and the budget left exceeds the
    expected compile latency (``jit_cost_s``, default: the measured average
    ``JIT_COMPILE_S``), compiles the JIT kernel on the engine's compile thread
    (``mg_jit_compile_async``) while the interpreter keeps scanning, then continues the
    SAME index stream on the compiled kernel.  Both kernels compute identical verdicts for
    every index (``tests/test_gpu_jit.py``), so the first hit does not depend on the mode.

    Launch sizes grow geometrically from ``chunk`` (easy queries answer in the first
    launch) and are capped by the measured rate so that a launch ends inside the budget
    (and inside ``max_launch_s``).  ``cancel`` (a ``threading.Event``) is checked before
    every launch: the hook sets it when z3 answered first (``plugin._race``).
    The model comes back with the hit (``mg_search``'s ``assign_out``)."""
    tp = time.perf_counter()
    P, blob = prepare(roots, gen)
    th = time.perf_counter()
    prog = engine.load(P.to_bytes())
    t0 = time.perf_counter()
    timing = {"host_prepare_ms": (th - tp) * 1e3}
    scanned = 0
    hit = None
    hits = 0
    used = "interp"
    expected_compile = JIT_COMPILE_S[0] if jit_cost_s is None else jit_cost_s
    expected_asm = JIT_ASM_COMPILE_S[0]
    assign = np.zeros(max(P.watch_words, 1), dtype=np.uint32) if want_model else None
    try:
        gh = engine.load_gen(prog, blob)
        timing["load_ms"] = (time.perf_counter() - th) * 1e3
        jh = None
        ticket = None      # the O3 kernel's compile
        ticket_asm = None  # the first tier's (assembly), submitted just before it
        tier = None        # "asm" / "o3": the compiled kernel in use
        asm_tried = o3_tried = False
        rate = None  # candidates/s of the kernel in use (last launch)
        last_n = 0   # candidates of the last launch
        race = None  # first tier vs O3: the first tier's handle and rate until the O3 kernel's first launch
        try:
            if jit == "always":
                tc = time.perf_counter()
                try:
                    jh = engine.jit_compile(prog, gh)
                    timing["jit_compile_ms"] = (time.perf_counter() - tc) * 1e3
                    used, tier = "jit", "o3"
                except Exception:  # the JIT rejected this program: scan on the interpreter
                    jit = "never"
            start = 0
            while scanned < max_candidates:
                now = time.perf_counter()
                left = timeout_s - (now - t0)
                if left <= 0 or (cancel is not None and cancel.is_set()):
                    break
                if ticket_asm is not None:
                    try:
                        h = engine.jit_poll(ticket_asm)
                    except Exception:  # outside the first tier: the interpreter until the O3 kernel
                        ticket_asm, h = None, None
                    if h is not None:
                        ticket_asm = None
                        took = now - tc
                        JIT_ASM_COMPILE_S[0] = 0.5 * JIT_ASM_COMPILE_S[0] + 0.5 * took
                        timing["jit_asm_compile_ms"] = took * 1e3
                        if jh is None:
                            jh, used, rate, tier = h, "jit", None, "asm"
                            timing["jit_switch_ms"] = (now - t0) * 1e3  # when the search moved to a kernel
                            timing["interp_candidates"] = scanned
                            chunk = max(chunk, 1 << 22)
                        else:
                            engine.jit_free(h)
                if ticket is not None:
                    try:
                        h = engine.jit_poll(ticket)
                    except Exception:  # JIT unavailable for this program: stay where we are
                        ticket, h = None, None
                        if jh is None:
                            jit = "never"
                    if h is not None:
                        ticket = None
                        if jh is not None:
                            # the O3 kernel takes over the same stream; the first tier's stays until one
                            # launch of the same size on the O3 kernel has shown which is faster (the first
                            # tier beats O3 on some queries: C2, profiles/r05f_tier_rates.jsonl)
                            race = {"asm_rate": rate, "n": last_n, "asm": jh}
                        else:
                            timing["jit_switch_ms"] = (now - t0) * 1e3
                            timing["interp_candidates"] = scanned
                        jh, used, rate, tier = h, "jit", None, "o3"
                        took = now - tc
                        timing["jit_compile_ms"] = took * 1e3
                        timing["o3_switch_ms"] = (now - t0) * 1e3
                        JIT_COMPILE_S[0] = 0.5 * JIT_COMPILE_S[0] + 0.5 * took
                        chunk = max(chunk, 1 << 22)
                # each tier is submitted at most once per search: a first tier that refused this
                # program (outside its vocabulary) is not asked again while the O3 kernel is not due
                want_asm = JIT_ASM and not asm_tried and left > 1.2 * expected_asm
                want_o3 = not o3_tried and left > 1.2 * expected_compile
                if (jh is None and ticket is None and ticket_asm is None and jit == "auto" and scanned > 0
                        and (want_asm or want_o3)):
                    tc = time.perf_counter()
                    if want_asm:
                        ticket_asm = engine.jit_compile_async(prog, gh, asm=True)
                        asm_tried = True
                    if want_o3:
                        ticket = engine.jit_compile_async(prog, gh)
                        o3_tried = True
                n = min(chunk, max_candidates - scanned)
                if race is not None and race["n"]:
                    n = min(n, race["n"])  # the race launch: as large as the first tier's last one
                if rate:
                    cap_s = left
                    if ticket is not None or ticket_asm is not None:
                        # 1-ms launches while the first tier is due (a few ms; measured cadence: a 10-ms
                        # launch started at 5 ms turned a 5.5-ms compile into a 15-ms switch)
                        short = now - tc < max(5 * JIT_FIRST_POLL_S,
                                               4 * expected_asm if ticket_asm is not None else 0.0)
                        cap_s = min(left, JIT_FIRST_POLL_S if short else JIT_POLL_S)
                    if max_launch_s is not None:
                        cap_s = min(cap_s, max_launch_s)
                    n = max(1, min(n, int(rate * cap_s)))
                tl = time.perf_counter()
                if jh is not None:
                    idx, nh = engine.jit_search(jh, seed, start, n, early_exit=True, assign=assign)
                else:
                    idx, nh = engine.search(prog, gh, seed, start, n, early_exit=True, assign=assign)
                dt = time.perf_counter() - tl
                last_n = n
                race_kept_asm = False
                if race is not None and jh is not None and tier == "o3":
                    o3_rate = n / dt if dt > 0 else 0.0
                    # the O3 rate is its module's first launch (start-up costs in it) and the first tier's
                    # came from another range: near-equal rates (within RACE_TIE) go to O3
                    keep_asm = bool(race["asm_rate"]) and o3_rate * (1.0 + RACE_TIE) < race["asm_rate"]
                    timing["tier_race"] = {"asm_rate": race["asm_rate"], "o3_rate": o3_rate, "n": n,
                                           "kept": "asm" if keep_asm else "o3"}
                    if keep_asm:
                        engine.jit_free(jh)
                        jh, tier = race["asm"], "asm"
                        race_kept_asm = True
                    else:
                        engine.jit_free(race["asm"])
                    race = None
                if ticket_asm is not None:  # the launches the first tier's compile waited behind
                    timing["asm_wait_launches"] = timing.get("asm_wait_launches", 0) + 1
                    timing["asm_wait_launch_max_ms"] = max(timing.get("asm_wait_launch_max_ms", 0.0), dt * 1e3)
                # the next launch is sized by the kernel that runs it: the first tier's own rate when the
                # race kept it (this launch's rate is the O3 kernel's)
                rate = timing["tier_race"]["asm_rate"] if race_kept_asm else (n / dt if dt > 0 else None)
                scanned += n
                start += n
                if idx is not None:
                    hit, hits = idx, nh
                    break
                # a first launch of 64 waves answers the easy queries in one program pass, and
                # with one group per block the engine captures the hit's model in the same pass
                # (mg_search); then geometric growth amortises the launch + sync per chunk
                # (x16 after the 2^12 capture launch: a query that misses there is not an easy one)
                chunk = min(chunk * (16 if chunk < (1 << 16) else 4), 1 << 26 if jh is None else 1 << 30)
        finally:
            if race is not None:
                engine.jit_free(race["asm"])
            if ticket_asm is not None:
                engine.jit_cancel(ticket_asm)
            if ticket is not None:
                engine.jit_cancel(ticket)
            if jh is not None:
                engine.jit_free(jh)
            engine.free_gen(gh)
    finally:
        engine.free(prog)
    dt = time.perf_counter() - t0
    res = SearchResult(hit, hits, scanned, dt)
    res.engine = used
    if tier is not None:
        timing["jit_tier"] = tier
    global LAST_ENGINE, LAST_RESULT
    LAST_ENGINE, LAST_RESULT = used, res
    if hit is not None and want_model:
        # the search only reports indices whose verdict is 1
        tm = time.perf_counter()
        res.model = (1,) + model_from_assignment(P, assign) + (P,)
        timing["model_ms"] = (time.perf_counter() - tm) * 1e3
    timing["search_ms"] = dt * 1e3
    res.timing = timing
    return res


def search_partitioned(engine, roots: Sequence[T.Term], timeout_s: float = 10.0, **kw) -> SearchResult:
    """Search each variable-disjoint bucket (``partition.py``) on its own and merge
    the bucket models (``independence_solver.py:119-140``).  ``index`` is the
    tuple of per-bucket first hits; the model tuple is
    ``(verdict, scalars, arrays, funcs, [programs])``."""
    from .partition import partition

    buckets = partition(roots)
    if len(buckets) <= 1:
        return search(engine, roots, timeout_s=timeout_s, **kw)
    t0 = time.perf_counter()
    idx, hits, scanned = [], 0, 0
    ver, scalars, arrays, funcs, progs = 1, {}, {}, {}, []
    engines = set()
    for b in buckets:
        left = timeout_s - (time.perf_counter() - t0)
        if left <= 0 or (kw.get("cancel") is not None and kw["cancel"].is_set()):
            res = SearchResult(None, 0, scanned, time.perf_counter() - t0)
            res.buckets = len(buckets)
            return res
        r = search(engine, b, timeout_s=left, **kw)
        scanned += r.scanned
        engines.add(getattr(r, "engine", "interp"))
        if r.index is None:
            res = SearchResult(None, 0, scanned, time.perf_counter() - t0)
            res.buckets = len(buckets)
            return res
        idx.append(r.index)
        hits += r.hits
        if r.model is not None:
            v, s_, a_, f_, p_ = r.model
            ver &= int(v)
            scalars.update(s_)
            arrays.update(a_)
            funcs.update(f_)
            progs.append(p_)
    res = SearchResult(tuple(idx), hits, scanned, time.perf_counter() - t0)
    res.buckets = len(buckets)
    res.engine = "+".join(sorted(engines))
    if kw.get("want_model", True):
        res.model = (ver, scalars, arrays, funcs, progs)
    return res


def eval_with_models(engine, P: ssa.Program, assigns: Sequence[Sequence[int]]):
    """Batched eval of explicit assignments; also reads every candidate back as a
    finite model ``(scalars, arrays, funcs)`` (site canonicalisation applied)."""
    entries, widths = model_watch(P)
    prev = P.watch
    P.set_watch(entries)
    soa = ssa.soa_from_assignments(P, assigns)
    prog = engine.load(P.to_bytes())
    try:
        ww = sum(ssa.limbs(w) for w in widths)
        ver, watch = engine.eval(prog, soa, len(assigns), watch_words=ww)
    finally:
        engine.free(prog)
        P.set_watch(prev)
    models = [decode_model(P, read_rows(watch, widths, i) if watch is not None else []) for i in range(len(assigns))]
    return ver, models
