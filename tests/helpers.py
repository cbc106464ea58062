"""Shared test infrastructure: golden-vector loaders, a random term-DAG
generator and the GPU-vs-oracle comparison used by the parity tests."""
from __future__ import annotations

import json
import random
from pathlib import Path
from typing import Dict, List, Sequence

import numpy as np

from mythril_amd import ssa
from mythril_amd.replay import ExceptionalHalt, ReplayUnsupported, replay, replay_assignment
from mythril_amd.smt import terms as T
from oracle.bv import OracleModel, evaluate_many

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_json(name):
    return json.loads((GOLDEN / name).read_text())


# VMTests vectors with a post-state that the replay refuses, by name: none since round 4
# (CALLDATACOPY, CODECOPY, SELFDESTRUCT and the input-dependent jumps of DynamicJump_value* and
# TestNameRegistrator, followed along the concrete path).  A regression that refuses more shows up
# as a failed assertion in vmtest_cases, not as a silently shorter list.
VMTEST_REFUSED: Dict[str, str] = {}


def vmtest_cases(follow: bool = True):
    """(name, vector, ReplayResult) for every VMTests vector whose outcome is a post-state (not
    ignored by the reference: ``tests/laser/evm_testsuite/evm_test.py:109-188``).  Input-dependent
    jumps are followed along the vector's concrete path (the oracle evaluates the decision; the
    replay keeps it as a path constraint, ``ReplayResult.path``)."""
    out, refused = [], {}
    for name, v in sorted(load_json("vmtests.json").items()):
        if v["reference_ignored"] or v["post_storage"] is None:
            continue
        pre = {int(k, 16): int(x, 16) for k, x in v["pre_storage"].items()}
        fol = None
        if follow:
            scal, arrs = replay_assignment(v)
            m = OracleModel(scal, arrs)
            fol = lambda t, m=m: evaluate_many([t], m)[0]  # noqa: E731
        try:
            r = replay(v["code"], bytes.fromhex(v["data"]), pre, follow=fol)
        except (ReplayUnsupported, ExceptionalHalt) as e:
            refused[name] = str(e)
            continue
        out.append((name, v, r))
    if follow:
        assert refused == VMTEST_REFUSED, f"replay refuses VMTests vectors: {refused}"
    return out


# ---------------------------------------------------------------------------
# random programs
# ---------------------------------------------------------------------------
EDGE_256 = [0, 1, 2, 3, 31, 32, 255, 256, 257, (1 << 255), (1 << 255) - 1, (1 << 256) - 1, (1 << 256) - 2,
            (1 << 128), (1 << 160) - 1, (1 << 64) + 1]

BIN_OPS = ["bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvand", "bvor",
           "bvxor", "bvshl", "bvlshr", "bvashr"]
CMP_OPS = ["bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge", "bvumul_noovfl"]


def edge_value(rng: random.Random, w: int) -> int:
    m = (1 << w) - 1
    r = rng.random()
    if r < 0.35:
        return rng.choice(EDGE_256) & m
    if r < 0.5:
        return rng.choice([0, 1, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1]) & m
    if r < 0.65:
        return rng.getrandbits(min(w, rng.choice([4, 8, 16, 64])))
    return rng.getrandbits(w)


class RandomProgram:
    """A random constraint DAG over scalars, one array and one UF, with a list of
    'interesting' terms to compare value-by-value."""

    def __init__(self, seed: int, n_ops: int = 40, widths=(256, 256, 256, 160, 64, 32, 8, 1 + 7, 257, 512)):
        rng = random.Random(seed)
        self.rng = rng
        self.vars: Dict[int, List[T.Term]] = {}
        pool: Dict[int, List[T.Term]] = {}

        def add(t):
            pool.setdefault(t.width, []).append(t)
            return t

        for i, w in enumerate(widths):
            v = T.BitVecVar(f"v{i}_{w}", w)
            self.vars.setdefault(w, []).append(v)
            add(v)
            add(T.BitVecVal(edge_value(rng, w), w))
        bools: List[T.Term] = [T.BoolVar("flag")]
        arr = T.ArrayVar("Storage", 256, 256)
        fn = T.FuncDecl("keccak256_512", 512, 256)
        terms: List[T.Term] = []
        for _ in range(n_ops):
            kind = rng.random()
            w = rng.choice([256, 256, 256, 64, 160, 8, 32])
            src = pool.get(w) or [T.BitVecVal(0, w)]
            a, b = rng.choice(src), rng.choice(src)
            if kind < 0.45:
                op = rng.choice(BIN_OPS)
                if op in ("bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvshl", "bvlshr", "bvashr") and w > 256:
                    op = "bvadd"
                t = T.bvbin(op, a, b)
            elif kind < 0.55:
                t = T.bvun(rng.choice(["bvnot", "bvneg"]), a)
            elif kind < 0.65:
                c = T.bvcmp(rng.choice(CMP_OPS), a, b) if w <= 256 else T.eq(a, b)
                bools.append(c)
                terms.append(c)
                continue
            elif kind < 0.72:
                c = rng.choice(bools)
                t = T.ite(c, a, b)
            elif kind < 0.80:
                hi = rng.randrange(w)
                lo = rng.randrange(hi + 1)
                t = T.extract(hi, lo, a)
            elif kind < 0.86:
                w2 = rng.choice([8, 32, 96, 160, 256])
                b2 = rng.choice(pool.get(w2) or [T.BitVecVal(1, w2)])
                t = T.concat(a, b2) if a.width + w2 <= 1024 else a
            elif kind < 0.90:
                k = rng.choice([1, 8, 96, 256])
                t = T.zero_extend(k, a) if rng.random() < 0.5 else T.sign_extend(k, a)
            elif kind < 0.95:
                idx = rng.choice(pool.get(256) or [T.BitVecVal(0, 256)])
                if rng.random() < 0.5:
                    st = T.store(arr, rng.choice(pool[256]), rng.choice(pool[256]))
                    t = T.select(st, idx)
                else:
                    t = T.select(arr, idx)
            else:
                x = rng.choice(pool.get(256))
                y = rng.choice(pool.get(256))
                t = T.app(fn, T.concat(x, y))
            add(t)
            terms.append(t)
        # logical glue
        for _ in range(4):
            x, y = rng.choice(bools), rng.choice(bools)
            c = rng.choice([T.and_(x, y), T.or_(x, y), T.not_(x), T.xor_(x, y), T.eq(x, y)])
            bools.append(c)
            terms.append(c)
        self.terms = terms
        self.bools = bools
        self.root = T.or_(*bools[-3:]) if len(bools) >= 3 else T.BoolVal(True)


def random_assignments(P: ssa.Program, n: int, seed: int):
    rng = random.Random(seed)
    return [[edge_value(rng, c.width) for c in P.coords] for _ in range(n)]


def lift_literals(terms: Sequence[T.Term], min_width: int = 8):
    """Replace every bit-vector literal (width >= min_width) by a fresh variable ``lit<k>``.
    Returns (new terms, {name: value}).  Evaluated with those values as runtime inputs, the
    JIT cannot constant-fold the arithmetic (hipRTC folds literal operands at -O3)."""
    memo: Dict[int, T.Term] = {}
    vals: Dict[str, int] = {}
    for t in T.postorder(list(terms)):
        if t.op == "bvconst" and t.width >= min_width:
            name = f"lit{len(vals)}_{t.width}"
            vals[name] = t.params[0]
            memo[t.id] = T.BitVecVar(name, t.width)
            continue
        args = tuple(memo[a.id] for a in t.args)
        memo[t.id] = t if args == t.args else T.mk(t.op, t.sort, args, t.params)
    return [memo[t.id] for t in terms], vals


def gpu_eval_terms(engine, roots: Sequence[T.Term], watch_terms: Sequence[T.Term], assigns=None, n=64, seed=0,
                   jit: bool = False, asm: bool = False, tiled: bool = False, o3: bool = False):
    """Evaluate on the GPU (the interpreter, or with ``jit`` the compiled eval kernel on the same
    runtime SoA inputs: with watch rows the first tier's by default, ``o3`` the O3 kernel); returns
    (P, assigns, verdicts, per-candidate dict term-id -> value, per-candidate oracle models)."""
    P = ssa.flatten(list(roots), extra=list(watch_terms))
    # watch every requested term that the program contains, plus the model read-back entries
    from mythril_amd.search import model_watch

    for t in watch_terms:
        if t.id not in P.term_node:
            raise KeyError("watch term not in program")
    term_entries = [P.term_node[t.id] for t in watch_terms]
    m_entries, m_widths = model_watch(P)
    entries = term_entries + m_entries
    widths = [P.node_width[e] for e in term_entries] + m_widths
    P.set_watch(entries)
    if assigns is None:
        assigns = random_assignments(P, n, seed)
    soa = ssa.soa_from_assignments(P, assigns)
    prog = engine.load(P.to_bytes())
    try:
        info = engine.info(prog)
        if jit or asm:
            jh = engine.jit_compile(prog, 0, asm=asm, tiled=tiled, o3=o3)
            try:
                from mythril_amd.native import tile_soa

                ver, watch = engine.jit_eval(jh, tile_soa(soa) if tiled else soa, len(assigns),
                                             watch_words=info.watch_words)
            finally:
                engine.jit_free(jh)
        else:
            ver, watch = engine.eval(prog, soa, len(assigns), watch_words=info.watch_words)
    finally:
        engine.free(prog)
    from mythril_amd.search import decode_model, read_rows

    results, models = [], []
    for i in range(len(assigns)):
        vals = read_rows(watch, widths, i)
        tv = {t.id: vals[j] for j, t in enumerate(watch_terms)}
        s, a, f = decode_model(P, vals[len(watch_terms):])
        results.append(tv)
        models.append(OracleModel(s, a, f))
    return P, assigns, ver, results, models


def literal_tail_query():
    """Mapping keys ``Concat(key, slot)`` with literal slots, as LASER addresses storage through
    ``keccak(Concat(key, slot))``: an EQ of an ITE over such keys, two keccak sites with slot 5 and
    one with slot 6 (different literal tails never compare equal)."""
    from mythril_amd.smt import Array, Concat, Function, If, Not, ULT, symbol_factory

    BVV, S = symbol_factory.BitVecVal, symbol_factory.BitVecSym
    a, b, d, e = S("nk_a", 256), S("nk_b", 256), S("nk_d", 256), S("nk_e", 256)
    slot, other = BVV(5, 256), BVV(6, 256)
    k1, k2, k3 = Concat(a, slot), Concat(b, slot), Concat(d, slot)
    h = Function("keccak256_512", 512, 256)
    storage = Array("Storage", 256, 256)
    return [If(ULT(a, b), k1, k2) == k3, Not(a == b),
            ULT(storage[h(k1)], storage[h(k3)] + BVV(3, 256)),
            Not(storage[h(Concat(e, other))] == BVV(0, 256))]


# operators of the first tier (random_tier_program)
_BIN = ["bvadd", "bvsub", "bvmul", "bvand", "bvor", "bvxor"]
_FULL_BIN = ["bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvshl", "bvlshr", "bvashr"]
_CMP = ["bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge", "bvumul_noovfl"]


def random_tier_program(seed: int, n_ops: int = 36, full: bool = False):
    """Random programs over the first tier's operators (``full``: also symbolic division, remainders,
    shifts, EXP and concrete Keccak): two ORs of random Bools, so verdicts carry information."""
    rng = random.Random(seed)
    pool = {}

    def add(t):
        pool.setdefault(t.width, []).append(t)
        return t

    for i, w in enumerate((256, 256, 160, 64, 32, 8, 1 + 7, 257, 512, 1)):
        if w == 1:
            continue
        add(T.BitVecVar(f"a{seed}_{i}_{w}", w))
        add(T.BitVecVal(edge_value(rng, w), w))
    bools = [T.BoolVar(f"f{seed}")]
    arr = T.ArrayVar("Storage", 256, 256)
    fn = T.FuncDecl("keccak256_512", 512, 256)
    for _ in range(n_ops):
        kind = rng.random()
        w = rng.choice([256, 256, 64, 160, 8, 32, 512])
        src = pool.get(w) or [T.BitVecVal(0, w)]
        a, b = rng.choice(src), rng.choice(src)
        if full and kind < 0.12:
            op = rng.choice(_FULL_BIN)
            t = T.bvbin(op, a, b) if w <= 256 else T.bvbin("bvadd", a, b)  # the lowering's bound
            if w <= 256 and op in ("bvshl", "bvlshr", "bvashr") and rng.random() < 0.6:  # amounts that matter
                t = T.bvbin(op, a, T.bvbin("bvand", b, T.BitVecVal(rng.choice([7, 63, 255, 511]), w)))
        elif full and kind < 0.16:
            t = T.bvexp(a, T.bvbin("bvand", b, T.BitVecVal(rng.choice([3, 15, 255]), w))) if w == 256 else a
        elif full and kind < 0.18 and w in (256, 512):
            t = T.keccak256(a)
        elif kind < 0.35:
            op = rng.choice(_BIN)
            t = T.bvbin(op if not (op == "bvmul" and w > 256) else "bvadd", a, b)
        elif kind < 0.45:
            t = T.bvun(rng.choice(["bvnot", "bvneg"]), a)
        elif kind < 0.60:
            c = T.bvcmp(rng.choice(_CMP), a, b) if w <= 256 else T.eq(a, b)
            bools.append(c)
            continue
        elif kind < 0.68:
            t = T.ite(rng.choice(bools), a, b)
        elif kind < 0.76:
            hi = rng.randrange(w)
            t = T.extract(hi, rng.randrange(hi + 1), a)
        elif kind < 0.82:
            w2 = rng.choice([8, 32, 96, 160, 256])
            b2 = rng.choice(pool.get(w2) or [T.BitVecVal(1, w2)])
            t = T.concat(a, b2) if a.width + w2 <= 1024 else a
        elif kind < 0.88:
            k = rng.choice([1, 8, 96, 256])
            t = T.zero_extend(k, a) if rng.random() < 0.5 else T.sign_extend(k, a)
        elif kind < 0.95:
            idx = rng.choice(pool[256])
            st = T.store(arr, rng.choice(pool[256]), rng.choice(pool[256])) if rng.random() < 0.5 else arr
            t = T.select(st, idx)
        else:
            t = T.app(fn, T.concat(rng.choice(pool[256]), rng.choice(pool[256])))
        add(t)
        if t.width <= 256 and rng.random() < 0.3:
            bools.append(T.eq(t, rng.choice(pool.get(t.width) or [t])))
    for _ in range(3):
        x, y = rng.choice(bools), rng.choice(bools)
        bools.append(rng.choice([T.and_(x, y), T.or_(x, y), T.not_(x), T.xor_(x, y), T.eq(x, y)]))
    # an OR of a few of them: satisfiable by many candidates, so verdicts carry information
    return [T.or_(*rng.sample(bools, min(3, len(bools)))), T.or_(*rng.sample(bools, min(3, len(bools))))]
