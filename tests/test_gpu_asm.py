"""The JIT's first tier (``jit_asm.cpp``: gfx950 assembly emitted by the engine, MG_JIT_ASM) against
the C port (``oracle/bveval.c``) on the same GEN3 candidate stream.

* per-candidate verdicts of the tier's ``mgj_gen`` on random unaligned 63-bit windows (two with bit
  31 of the low index word set), for every workload inside the tier, the bench's hard needle, the
  literal-tail mapping keys and random programs over the tier's operators;
* its ``mgj_search``: first hit and hit count of each window equal the C port's, and an early-exit
  search from index 0 finds the same first hit as the O3 kernel and the interpreter;
* the full-size property: the hard needle (~2^-24, first hit near index 3.2e8) found at the same
  index by the tier and by the O3 kernel.

Reference anchor: a candidate's verdict is ``Model.eval(And(constraints), model_completion=True)``
(``mythril/laser/smt/model.py:45-59``) of the query ``get_model`` receives
(``mythril/support/model.py:15-49``).
"""
import random
import zlib

import numpy as np
import pytest

from mythril_amd import native, search, workloads
from mythril_amd.smt import terms as T

pytestmark = pytest.mark.gpu

N = 2048
OUTSIDE = set()  # since round 5 the tier takes Keccak, EXP, signed / symbolic division and variable shifts


def _windows(rng, k=4):
    out = []
    for w in range(k):
        start = rng.getrandbits(63)
        if w < 2:
            start = (start & ~0xFFFFFFFF) | 0x80000000 | rng.getrandbits(31)
        out.append(start | 1)
    return out


def _check(engine, name, roots, seeds=2, windows=4):
    from oracle import cport

    rng = random.Random(zlib.crc32(name.encode()) ^ 0x61736D)
    P, blob = search.prepare(roots)
    pb = P.to_bytes()
    prog = engine.load(pb)
    gh = engine.load_gen(prog, blob)
    ja = engine.jit_compile(prog, gh, gen_verdicts=True, asm=True)
    try:
        for _ in range(seeds):
            seed = rng.getrandbits(32)
            for start in _windows(rng, windows):
                cf, ch, want = cport.search(pb, blob, seed, start, N, threads=16, verdicts=True)
                va = engine.jit_verdicts(ja, seed, start, N)
                bad = np.nonzero(va != want)[0]
                assert bad.size == 0, (f"{name}: asm tier {bad.size} mismatches, first at index {start + int(bad[0])} "
                                       f"seed {seed} (asm {va[bad[0]]}, C port {want[bad[0]]})")
                assert engine.jit_search(ja, seed, start, N, early_exit=False) == (cf, ch)
                ef, _ = engine.jit_search(ja, seed, start, N, early_exit=True)
                assert ef == cf
    finally:
        engine.jit_free(ja)
        engine.free_gen(gh)
        engine.free(prog)


def _queries():
    from tests.helpers import literal_tail_query
    import bench

    q = {n: (lambda n=n: [c.raw for c in workloads.WORKLOADS[n]()]) for n in sorted(workloads.WORKLOADS)
         if n not in OUTSIDE}
    q["hard_needle"] = lambda: bench.hard_query(workloads.WORKLOADS["token_transfer_underflow"]())
    q["literal_tail_keys"] = lambda: [c.raw for c in literal_tail_query()]
    return q


@pytest.mark.parametrize("name", sorted(_queries()))
def test_asm_tier_verdicts(engine, name):
    _check(engine, name, _queries()[name]())


def _random_program(seed: int, n_ops: int = 36, full: bool = False):
    from tests.helpers import random_tier_program

    return random_tier_program(seed, n_ops, full=full)


# 200 random programs (8 chunks of 25), every other one over the full vocabulary (symbolic
# division and remainders, signed division, variable shifts, EXP, Keccak)
@pytest.mark.parametrize("chunk", range(8))
def test_asm_tier_random_programs(engine, chunk):
    for k in range(25):
        seed = 1000 + 25 * chunk + k
        roots = _random_program(seed, full=bool(k & 1))
        P, blob = search.prepare(roots)
        native.jit_asm(P.to_bytes(), blob)  # inside the tier (raises otherwise)
        _check(engine, f"random{seed}", roots, seeds=1, windows=2)


def test_asm_tier_first_hit_from_zero(engine):
    """Early-exit searches from index 0 (the product's shape): the tier, the O3 kernel and the
    interpreter report the same first hit on every workload inside the tier."""
    for name in sorted(workloads.WORKLOADS):
        if name in OUTSIDE:
            continue
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        prog = engine.load(P.to_bytes())
        gh = engine.load_gen(prog, blob)
        ja = engine.jit_compile(prog, gh, asm=True)
        jo = engine.jit_compile(prog, gh)
        try:
            for count in (1 << 12, 1 << 20):
                a = engine.jit_search(ja, 7, 0, count, early_exit=True)[0]
                o = engine.jit_search(jo, 7, 0, count, early_exit=True)[0]
                i = engine.search(prog, gh, 7, 0, count, early_exit=True)[0]
                assert a == o == i, (name, count, a, o, i)
        finally:
            engine.jit_free(ja)
            engine.jit_free(jo)
            engine.free_gen(gh)
            engine.free(prog)


def test_asm_tier_hard_needle_full_size(engine):
    """The bench's hard query at full size: the ~2^-24 needle near index 3.2e8, found at the same
    index by the tier and by the O3 kernel (hit counts over the whole sweep agree too)."""
    import bench

    roots = bench.hard_query(workloads.WORKLOADS["token_transfer_underflow"]())
    P, blob = search.prepare(roots)
    prog = engine.load(P.to_bytes())
    gh = engine.load_gen(prog, blob)
    ja = engine.jit_compile(prog, gh, asm=True)
    jo = engine.jit_compile(prog, gh)
    try:
        seed = 0x6D797468
        n = 1 << 29
        fa, ha = engine.jit_search(ja, seed, 0, n, early_exit=False)
        fo, ho = engine.jit_search(jo, seed, 0, n, early_exit=False)
        assert (fa, ha) == (fo, ho) and fa is not None
        assert engine.jit_search(ja, seed, 0, n, early_exit=True)[0] == fa
    finally:
        engine.jit_free(ja)
        engine.jit_free(jo)
        engine.free_gen(gh)
        engine.free(prog)


# ---------------------------------------------------------------------------------------------
# the first tier's eval kernel (mgj_eval from jit_asm.cpp): explicit SoA coordinates, watch rows
# ---------------------------------------------------------------------------------------------
# model read-back on the tier's eval kernel: 200 random programs (8 chunks of 25), watch rows
@pytest.mark.parametrize("chunk", range(8))
def test_asm_eval_random_programs_terms(engine, chunk):
    for k in range(25):
        _eval_terms(engine, 25 * chunk + k, tiled=bool(k % 3 == 0), n=48, full=bool(k & 1))


def _eval_terms(engine, seed, tiled, n=200, full=False):
    """``Model.eval`` batched on the first tier's eval kernel: every watched term's value and every
    verdict equal the Python oracle's on edge-value assignments (``oracle/bv.py``, the reference's
    ``model.eval(..., model_completion=True)``), as the O3 eval kernel's do."""
    from tests.helpers import gpu_eval_terms
    from oracle.bv import evaluate_many

    roots = _random_program(3000 + seed, full=full)
    P0, _ = search.prepare(roots)
    native.jit_asm(P0.to_bytes(), None)  # inside the tier (raises otherwise)
    watch = [t for t in T.postorder(roots) if t.sort[0] == "bv"][:24]
    P, assigns, ver, vals, models = gpu_eval_terms(engine, roots, watch, n=n, seed=seed, asm=True, tiled=tiled)
    for i, m in enumerate(models):
        want = evaluate_many(list(roots) + watch, m)
        assert ver[i] == int(all(want[:len(roots)])), (seed, i)
        for k, t in enumerate(watch):
            assert vals[i][t.id] == want[len(roots) + k], (seed, i, k)


@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("n", [5000 + 37, (1 << 18) + 37])
@pytest.mark.parametrize("name", ["token_transfer_underflow", "suicide_kill", "etherstore_reentrancy",
                                  "walletlibrary_kill"])
def test_asm_eval_workload_verdicts(engine, name, n, tiled):
    """The unspecialised workload program on random SoA rows: the first tier's eval verdicts equal
    the C port's (``oracle/bveval.c`` eval) and the O3 eval kernel's, at an n that leaves a partial
    last wave; at 2^18 + 37 every wave sweeps several groups, so the next group's rows loaded while
    the current group finishes (the cross-group row ring) are exercised.  ``tiled``: both kernels
    compiled for the tiled SoA (MG_JIT_SOA_TILED) read the same data re-laid (native.tile_soa),
    against the C port on the row-major original."""
    from oracle import cport

    P, _ = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
    # the verdicts-only program; search.prepare's Program is the flatten cache's, so its watch list
    # (the model read-back rows later searches of this workload decode) is put back
    prev = P.watch
    P.set_watch([])
    pb = P.to_bytes()
    P.set_watch(prev)
    prog = engine.load(pb)
    info = engine.info(prog)
    rng = np.random.default_rng(7)
    soa = rng.integers(0, 1 << 32, size=(int(info.coord_words), n), dtype=np.uint64).astype(np.uint32)
    # mask each coordinate row to its width (the layout mg_eval expects)
    from mythril_amd import ssa

    offs = P.coord_row_offsets()
    for c in P.coords:
        for j in range(ssa.limbs(c.width)):
            bits = min(32, c.width - 32 * j)
            soa[offs[c.index] + j] &= np.uint32((1 << bits) - 1)
    ja = engine.jit_compile(prog, 0, asm=True, tiled=tiled)
    jo = engine.jit_compile(prog, 0, tiled=tiled)
    src = native.tile_soa(soa) if tiled else soa
    try:
        va, _ = engine.jit_eval(ja, src, n)
        vo, _ = engine.jit_eval(jo, src, n)
    finally:
        engine.jit_free(ja)
        engine.jit_free(jo)
        engine.free(prog)
    want = cport.eval_soa(pb, soa, n)
    assert np.array_equal(va, want) and np.array_equal(vo, want)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 200])
def test_eval_tiled_small_n(engine, n):
    """The tiled SoA at sizes around one 64-candidate block (the last block padded): both eval
    kernels' verdicts equal the C port's on the row-major original."""
    from oracle import cport
    from mythril_amd import ssa

    P, _ = search.prepare([c.raw for c in workloads.WORKLOADS["suicide_kill"]()])
    prev = P.watch
    P.set_watch([])
    pb = P.to_bytes()
    P.set_watch(prev)
    prog = engine.load(pb)
    info = engine.info(prog)
    rng = np.random.default_rng(n)
    soa = rng.integers(0, 1 << 32, size=(int(info.coord_words), n), dtype=np.uint64).astype(np.uint32)
    offs = P.coord_row_offsets()
    for c in P.coords:
        for j in range(ssa.limbs(c.width)):
            bits = min(32, c.width - 32 * j)
            soa[offs[c.index] + j] &= np.uint32((1 << bits) - 1)
    want = cport.eval_soa(pb, soa, n)
    try:
        for asm in (False, True):
            jh = engine.jit_compile(prog, 0, asm=asm, tiled=True)
            try:
                v, _ = engine.jit_eval(jh, native.tile_soa(soa), n)
            finally:
                engine.jit_free(jh)
            assert np.array_equal(v, want), (asm, n)
    finally:
        engine.free(prog)


@pytest.mark.parametrize("wa", [8, 32, 64, 160, 256])
def test_asm_tier_umul_noovf(engine, wa):
    """bvumul_noovfl at several widths on the first tier: per-candidate verdicts equal the C port's
    (the generator's small, dictionary and uniform draws give products on both sides of 2^wa)."""
    x, y = T.BitVecVar(f"mx{wa}", wa), T.BitVecVar(f"my{wa}", wa)
    z = T.BitVecVar(f"mz{wa}", wa)
    roots = [T.or_(T.bvcmp("bvumul_noovfl", x, y), T.bvcmp("bvumul_noovfl", z, T.BitVecVal(3, wa)))]
    _check(engine, f"umul{wa}", roots, seeds=2, windows=3)
