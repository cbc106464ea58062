"""GPU parity of the JIT-specialised kernels (hipRTC) against the interpreter
kernels and the C restatement — bit-exact verdicts, per-term values, first hits."""
import random

import numpy as np
import pytest

from helpers import RandomProgram, load_json, random_assignments, vmtest_cases
from mythril_amd import native, search, ssa, workloads
from mythril_amd.replay import replay_assignment
from mythril_amd.smt import terms as T
from oracle.bv import OracleModel, evaluate

pytestmark = pytest.mark.gpu


def _eval_both(engine, P, assigns, o3=False):
    """The interpreter's and a compiled eval kernel's verdicts and watch rows on the same SoA (with
    watch rows the compiled kernel is the first tier's by default, ``o3``: the O3 kernel)."""
    soa = ssa.soa_from_assignments(P, assigns)
    prog = engine.load(P.to_bytes())
    try:
        info = engine.info(prog)
        v_i, w_i = engine.eval(prog, soa, len(assigns), watch_words=info.watch_words)
        jit = engine.jit_compile(prog, 0, o3=o3)
        try:
            v_j, w_j = engine.jit_eval(jit, soa, len(assigns), watch_words=info.watch_words)
        finally:
            engine.jit_free(jit)
    finally:
        engine.free(prog)
    return v_i, w_i, v_j, w_j


@pytest.mark.parametrize("o3", [False, True], ids=["default", "o3"])
@pytest.mark.parametrize("seed", range(6))
def test_jit_eval_matches_interpreter_random_dags(engine, seed, o3):
    rp = RandomProgram(500 + seed, n_ops=60)
    P = ssa.flatten([rp.root], extra=rp.terms)
    from mythril_amd.search import model_watch

    ent, _ = model_watch(P)
    P.set_watch([P.term_node[t.id] for t in rp.terms] + ent)
    assigns = random_assignments(P, 256, seed)
    v_i, w_i, v_j, w_j = _eval_both(engine, P, assigns)
    assert (v_i == v_j).all()
    assert (w_i == w_j).all()


def test_jit_eval_vmtests_sample(engine):
    """A sample of VMTests replay programs (incl. SHA3 and EXP) through the JIT eval kernel."""
    cases = vmtest_cases()
    rng = random.Random(5)
    pick = [c for c in cases if c[1]["dir"] == "vmSha3Test"] + rng.sample(cases, 16)
    for name, v, r in pick:
        keys = [int(k, 16) for k in v["post_storage"]]
        if not keys:
            continue
        words = [r.storage_word(k).raw for k in keys]
        P = ssa.flatten([T.BoolVal(True)], extra=words)
        P.set_watch([P.term_node[w.id] for w in words])
        scal, arrs = replay_assignment(v)
        m = OracleModel(scal, arrs)
        assign = [0] * len(P.coords)
        for c in P.coords:
            if c.kind == ssa.COORD_SCALAR:
                assign[c.index] = scal.get(c.name, 0)
            else:
                key = evaluate(P.node_term[P.site_key_node[c.index]], m)
                assign[c.index] = arrs.get(c.name, ({}, 0))[0].get(key, 0)
        v_i, w_i, v_j, w_j = _eval_both(engine, P, [assign])
        row = 0
        for k, x in v["post_storage"].items():
            assert ssa.limbs_to_int(w_j[row:row + 8, 0]) == int(x, 16), (name, k)
            row += 8


@pytest.mark.parametrize("aux", [False, True])
@pytest.mark.parametrize("shaped", [False, True])
@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS), ids=workloads.test_id)
def test_jit_search_matches_interpreter_and_c(engine, name, shaped, aux):
    from oracle import cport

    roots = [c.raw for c in workloads.WORKLOADS[name]()]
    P = ssa.flatten(roots, aux_words=aux)
    blob = search.default_generator(P, roots=roots if shaped else None).blob()
    prog = engine.load(P.to_bytes())
    gh = engine.load_gen(prog, blob)
    jit = engine.jit_compile(prog, gh, gen_verdicts=True)
    try:
        for start, n in ((0, 1 << 12), (987654321, 1 << 16)):
            a = engine.search(prog, gh, 77, start, n, early_exit=False)
            b = engine.jit_search(jit, 77, start, n, early_exit=False)
            assert a == b, (start, a, b)
        c = cport.search(P.to_bytes(), blob, 77, 0, 1 << 12, threads=8)[:2]
        assert c == engine.jit_search(jit, 77, 0, 1 << 12, early_exit=False)
        # per-candidate verdicts: JIT (through the hit stream of unaligned 1-candidate windows is
        # too slow) -- compare the C port's verdict vector with the interpreter's GEN-mode verdicts
        cf, ch, cver = cport.search(P.to_bytes(), blob, 77, 4096 + 13, 3000, threads=8, verdicts=True)
        gver, _ = engine.eval_generated(prog, gh, 77, 4096 + 13, 3000)
        assert (gver == cver).all(), int((gver != cver).sum())
        # the JIT kernel candidate by candidate (mgj_gen: the same specialised body as mgj_search)
        jver = engine.jit_verdicts(jit, 77, 4096 + 13, 3000)
        assert (jver == cver).all(), int((jver != cver).sum())
        assert (cf, ch) == engine.jit_search(jit, 77, 4096 + 13, 3000, early_exit=False)
        # early exit keeps the exact first hit
        full = engine.jit_search(jit, 77, 0, 1 << 20, early_exit=False)[0]
        fast = engine.jit_search(jit, 77, 0, 1 << 20, early_exit=True)[0]
        assert full == fast
    finally:
        engine.jit_free(jit)
        engine.free_gen(gh)
        engine.free(prog)


def test_jit_edge_arithmetic_runtime_operands(engine):
    """Every binary op over the 256-bit edge set through the JIT eval kernel, operands as
    runtime SoA inputs (nothing for hipRTC to fold), bit-exact against the oracle."""
    from helpers import BIN_OPS, CMP_OPS, EDGE_256, gpu_eval_terms

    a = T.BitVecVar("a", 256)
    b = T.BitVecVar("b", 256)
    terms = [T.bvbin(op, a, b) for op in BIN_OPS] + [T.bvcmp(op, a, b) for op in CMP_OPS] + \
            [T.bvun("bvneg", a), T.bvun("bvnot", a), T.bvexp(a, b)]
    vals = EDGE_256 + [(1 << 256) - 5, 3 << 254, 0x1234567890ABCDEF << 100, 7]
    assigns = [[x, y] for x in vals for y in vals]
    P, _, ver, got, models = gpu_eval_terms(engine, [T.BoolVal(True)], terms, assigns, jit=True)
    for i, (x, y) in enumerate(assigns):
        want = evaluate_many_terms(terms, {"a": x, "b": y})
        for t, w in zip(terms, want):
            assert got[i][t.id] == w, (t.op, hex(x), hex(y))


def test_jit_narrow_widths_runtime_operands(engine):
    from helpers import gpu_eval_terms

    rng = random.Random(3)
    for w in (1, 7, 8, 31, 32, 33, 63, 64, 65, 100, 160, 255):
        a = T.BitVecVar("a", w)
        b = T.BitVecVar("b", w)
        terms = [T.bvbin(op, a, b) for op in ["bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem",
                                              "bvsmod", "bvshl", "bvlshr", "bvashr", "bvand", "bvor", "bvxor"]]
        terms += [T.bvcmp(op, a, b) for op in ["bvult", "bvule", "bvslt", "bvsle", "bvumul_noovfl"]]
        terms += [T.zero_extend(5, a), T.sign_extend(40, a), T.concat(a, b), T.extract(w - 1, w // 2, a)]
        m = (1 << w) - 1
        assigns = [[rng.choice([0, 1, m, m >> 1, (m >> 1) + 1, rng.getrandbits(w)]),
                    rng.choice([0, 1, m, m >> 1, (m >> 1) + 1, rng.getrandbits(w), w, w - 1])] for _ in range(64)]
        P, _, ver, got, models = gpu_eval_terms(engine, [T.BoolVal(True)], terms, assigns, jit=True)
        for i, (x, y) in enumerate(assigns):
            want = evaluate_many_terms(terms, {"a": x, "b": y})
            for t, wv in zip(terms, want):
                assert got[i][t.id] == wv, (w, t.op, x, y)


def test_jit_vmtests_literals_as_runtime_inputs(engine):
    """VMTests replay programs through the JIT eval kernel with every PUSH literal lifted
    into a runtime coordinate (tests/laser/evm_testsuite/evm_test.py:109-188 post-states):
    this checks the kernel's arithmetic, not hipRTC's constant folder.  Every vector on the default
    watch-row kernel (the first tier's since round 5: EXP, Keccak, signed and symbolic division,
    variable shifts included); `test_jit_vmtests_o3_sample` runs every sixth on the O3 kernel."""
    _vmtests_replay(engine, o3=False)


@pytest.mark.gpu
def test_jit_vmtests_o3_sample(engine):
    """Every sixth VMTests vector of the replay above on the O3 watch-row kernel (MG_JIT_O3)."""
    _vmtests_replay(engine, o3=True)


def _vmtests_replay(engine, o3):
    from helpers import lift_literals

    cases = vmtest_cases()
    checked = 0
    for ci, (name, v, r) in enumerate(cases):
        keys = [int(k, 16) for k in v["post_storage"]]
        if not keys or (o3 and ci % 6):
            continue
        words = [r.storage_word(k).raw for k in keys]
        lifted, lits = lift_literals(words)
        P = ssa.flatten([T.BoolVal(True)], extra=lifted)
        P.set_watch([P.term_node[w.id] for w in lifted])
        scal, arrs = replay_assignment(v)
        scal = dict(scal, **lits)
        m = OracleModel(scal, arrs)
        assign = [0] * len(P.coords)
        for c in P.coords:
            if c.kind == ssa.COORD_SCALAR:
                assign[c.index] = scal.get(c.name, 0)
            else:
                key = evaluate(P.node_term[P.site_key_node[c.index]], m)
                assign[c.index] = arrs.get(c.name, ({}, 0))[0].get(key, 0)
        soa = ssa.soa_from_assignments(P, [assign])
        prog = engine.load(P.to_bytes())
        try:
            info = engine.info(prog)
            jh = engine.jit_compile(prog, 0, o3=o3)
            try:
                flags, _, _ = engine.jit_layout(jh)
                # round 6: every read-back is inside the first tier (the three with 63 live keys run
                # `solo`), so none pays the O3 compile; the O3 sample asks for O3 explicitly
                assert bool(flags & native.MG_JIT_ASM) == (not o3), (name, flags)
                _, w_j = engine.jit_eval(jh, soa, 1, watch_words=info.watch_words)
            finally:
                engine.jit_free(jh)
        finally:
            engine.free(prog)
        row = 0
        for k, x in v["post_storage"].items():
            assert ssa.limbs_to_int(w_j[row:row + 8, 0]) == int(x, 16), (name, k)
            row += 8
        checked += len(v["post_storage"])
    assert checked >= (60 if o3 else 390)


def evaluate_many_terms(terms, scalars):
    from oracle.bv import evaluate_many

    return evaluate_many(terms, OracleModel(scalars))


@pytest.mark.gpu
def test_jit_verdicts_at_high_indices():
    """Per-candidate JIT verdicts against the C port on windows whose group bases have bit 31 of
    the low word set, and near 2^63 (64-bit index handling in the kernel prologue)."""
    from mythril_amd import native, search, workloads
    from oracle import cport

    eng = native.Engine.get()
    for name in ("token_transfer_underflow", "etherstore_reentrancy", "bectoken_batch_overflow"):
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        prog = eng.load(P.to_bytes())
        gh = eng.load_gen(prog, blob)
        jh = eng.jit_compile(prog, gh, gen_verdicts=True)
        try:
            for start in ((1 << 31) - 100, (1 << 40) | 0x80000013, (1 << 63) | 0xFFFFF000, (1 << 62) + 0x9ABCDEF1):
                _, _, want = cport.search(P.to_bytes(), blob, 0x5EED, start, 1500, threads=8, verdicts=True)
                got = eng.jit_verdicts(jh, 0x5EED, start, 1500)
                assert np.array_equal(got, want), (name, hex(start))
        finally:
            eng.jit_free(jh)
            eng.free_gen(gh)
            eng.free(prog)


@pytest.mark.parametrize("name", ["suicide_kill", "bectoken_batch_overflow"], ids=workloads.test_id)
def test_hit_counts_over_many_blocks(engine, name):
    """A launch of hundreds of blocks: the hit count is summed on the host from 16 count stripes
    (engine.hip kHitStripes) and the first hit is the minimum over every block's publish — both must
    equal the C port's over the same 2^18 candidates, for the compiled kernel and the interpreter."""
    from oracle import cport

    roots = [c.raw for c in workloads.WORKLOADS[name]()]
    P, blob = search.prepare(roots)
    prog = engine.load(P.to_bytes())
    gh = engine.load_gen(prog, blob)
    jit = engine.jit_compile(prog, gh)
    try:
        start, n = (1 << 40) + 12345, 1 << 18
        want = cport.search(P.to_bytes(), blob, 5, start, n, threads=16)[:2]
        assert want[1] > 0
        assert engine.jit_search(jit, 5, start, n, early_exit=False) == want
        assert engine.search(prog, gh, 5, start, n, early_exit=False) == want
    finally:
        engine.jit_free(jit)
        engine.free_gen(gh)
        engine.free(prog)


@pytest.mark.parametrize("seed", range(6))
def test_jit_eval_without_watch_rows_random_dags(engine, seed):
    """A program without watch rows gets the eval kernel whose SoA loads walk the rows with one
    pointer (jit.cpp K_COORD): its verdicts equal the interpreter's on the same SoA."""
    rp = RandomProgram(700 + seed, n_ops=60)
    P = ssa.flatten([rp.root])
    assert not P.watch
    assigns = random_assignments(P, 512, seed)
    v_i, _, v_j, _ = _eval_both(engine, P, assigns)
    assert (v_i == v_j).all()


@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS))
def test_jit_eval_without_watch_rows_workloads(engine, name):
    """The bench's roofline_eval program (every BASELINE workload, model watch dropped): JIT eval
    verdicts equal the interpreter's over edge-value assignments."""
    P, _ = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
    prev = P.watch
    P.set_watch([])
    try:
        assigns = random_assignments(P, 256, 11)
        v_i, _, v_j, _ = _eval_both(engine, P, assigns)
    finally:
        P.set_watch(prev)
    assert (v_i == v_j).all()
