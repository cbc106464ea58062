"""GPU parity: the HIP engine vs the oracle, bit-exact (integer/byte work).

Every test calls through the C-ABI (libmythgpu.so via ctypes).  Reference
anchors: VMTests post-states (evm_test.py:109-188), EIP-145 vectors
(tests/instructions/{shl,shr,sar}_test.py), Keccak KATs, the UF-keccak verdicts
of tests/laser/keccak_tests.py:7-138, and z3 model.eval semantics restated in
oracle/bv.py for random DAGs.
"""
import random

import numpy as np
import pytest

from helpers import RandomProgram, gpu_eval_terms, load_json, random_assignments, vmtest_cases
from mythril_amd import search, ssa, workloads
from mythril_amd.replay import replay_assignment
from mythril_amd.smt import (And, Array, BVMulNoOverflow, Concat, Function, LShR, Not, UGE, UGT, ULT,
                             symbol_factory)
from mythril_amd.smt import terms as T
from oracle.bv import OracleModel, evaluate, evaluate_many
from oracle.keccak import keccak256

pytestmark = pytest.mark.gpu
BVV = symbol_factory.BitVecVal


def test_keccak_batch(engine):
    rng = random.Random(7)
    lens = [0, 1, 2, 5, 10, 31, 32, 33, 64, 135, 136, 137, 200, 271, 272, 273, 1000] + [rng.randrange(0, 600) for _ in range(200)]
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in lens]
    got = engine.keccak256(msgs)
    for m, g in zip(msgs, got):
        assert g == keccak256(m), len(m)
    # KATs
    for kat in load_json("keccak_kat.json"):
        d = engine.keccak256([bytes.fromhex(kat["msg_hex"])])[0]
        if "digest" in kat:
            assert "0x" + d.hex() == kat["digest"]
        else:
            assert "0x" + d[:4].hex() == kat["selector"]


def test_vmtests_replay_on_gpu(engine):
    """Concrete replay programs of every covered VMTests vector, evaluated on the GPU,
    reproduce the expected post-state storage words."""
    cases = vmtest_cases()
    assert len(cases) == 429  # every non-ignored vector with a post-state (helpers.VMTEST_REFUSED)
    checked = 0
    for name, v, r in cases:
        keys = [int(k, 16) for k in v["post_storage"]]
        if not keys:
            continue
        words = [r.storage_word(k).raw for k in keys]
        truth = T.BoolVal(True)
        # the path constraints of followed jumps are the query: they must hold (verdict 1)
        P = ssa.flatten([truth] + list(r.path) + [T.eq(w, w) for w in words])
        P.set_watch([P.term_node[w.id] for w in words])
        scal, arrs = replay_assignment(v)
        assign = []
        for c in P.coords:
            if c.kind == ssa.COORD_SCALAR:
                assign.append(scal.get(c.name, 0))
            else:  # calldata[...] site: the byte at that index
                assign.append(None)
        # site coordinates need the concrete byte at the site's index: evaluate the key with the oracle
        m = OracleModel(scal, arrs)
        for c in P.sites:
            key = evaluate(P.node_term[P.site_key_node[c.index]], m)
            table, dflt = arrs.get(c.name, ({}, 0))
            assign[c.index] = table.get(key, dflt)
        soa = ssa.soa_from_assignments(P, [assign])
        prog = engine.load(P.to_bytes())
        try:
            info = engine.info(prog)
            ver, watch = engine.eval(prog, soa, 1, watch_words=info.watch_words)
        finally:
            engine.free(prog)
        assert ver[0] == 1
        row = 0
        for k, x in v["post_storage"].items():
            val = ssa.limbs_to_int(watch[row:row + 8, 0])
            row += 8
            assert val == int(x, 16), (name, k)
            checked += 1
    assert checked >= 390


def test_vmtests_jumps_followed_on_gpu(engine):
    """The vectors whose jumps depend on calldata (DynamicJump_value*, TestNameRegistrator), followed
    through the product path: ``replay.engine_follow`` evaluates every decision on the GPU, and the
    replay takes the same branches and keeps the same path constraints as with the oracle."""
    from mythril_amd.replay import engine_follow, replay

    n = 0
    for name, v, r in vmtest_cases():
        if not r.path:
            continue
        scal, arrs = replay_assignment(v)
        pre = {int(k, 16): int(x, 16) for k, x in v["pre_storage"].items()}
        r2 = replay(v["code"], bytes.fromhex(v["data"]), pre, follow=engine_follow(engine, scal, arrs))
        assert [T.to_sexpr(t) for t in r2.path] == [T.to_sexpr(t) for t in r.path], name
        assert r2.halted == r.halted
        n += 1
    assert n >= 4


@pytest.mark.parametrize("op", ["shl", "shr", "sar"])
def test_eip145_on_gpu(engine, op):
    rows = load_json("eip145.json")[op]
    value = symbol_factory.BitVecSym("value", 256)
    shift = symbol_factory.BitVecSym("shift", 256)
    term = {"shl": value << shift, "shr": LShR(value, shift), "sar": value >> shift}[op]
    assigns = [[int(r["value"], 16), int(r["shift"], 16)] for r in rows]
    P, _, ver, vals, _ = gpu_eval_terms(engine, [T.BoolVal(True), T.eq(term.raw, term.raw)], [term.raw], assigns)
    assert [c.name for c in P.coords] == ["value", "shift"]
    for r, tv in zip(rows, vals):
        assert tv[term.raw.id] == int(r["expected"], 16), r


@pytest.mark.parametrize("seed", range(12))
def test_random_dags_bit_exact(engine, seed):
    """Random DAGs over widths 1..1024 incl. arrays/UFs: every term, every candidate,
    bit-exact against the oracle under the model the GPU read back."""
    rp = RandomProgram(seed, n_ops=60)
    watch = [t for t in rp.terms]
    P, assigns, ver, vals, models = gpu_eval_terms(engine, [rp.root], watch, n=96, seed=1000 + seed)
    for i in range(len(assigns)):
        m = models[i]
        # scalar coordinates read back == what we supplied
        for c in P.scalar_coords():
            assert m.scalars[c.name] == assigns[i][c.index] & ((1 << c.width) - 1)
        memo = {}
        want = evaluate_many(watch + [rp.root], m, memo)
        for t, w in zip(watch, want):
            assert vals[i][t.id] == w, (seed, i, T.to_sexpr(t, 2))
        assert ver[i] == want[-1]
        # canonicalisation: the first site of a table to see a key takes its own
        # coordinate (later sites with an equal key reuse it — checked above via
        # the select/app term values)
        seen = set()
        for c in P.sites:
            key = evaluate(P.node_term[P.site_key_node[c.index]], m, memo)
            if (c.kind, c.name, key) in seen:
                continue
            seen.add((c.kind, c.name, key))
            table = (m.arrays if c.kind == ssa.COORD_ARRAY_SITE else m.funcs)[c.name][0]
            assert table[key] == assigns[i][c.index] & ((1 << c.width) - 1)


def test_edge_arithmetic_exhaustive(engine):
    """All binary ops over the 256-bit edge set (cross product), bit-exact."""
    from helpers import BIN_OPS, CMP_OPS, EDGE_256

    a = T.BitVecVar("a", 256)
    b = T.BitVecVar("b", 256)
    terms = [T.bvbin(op, a, b) for op in BIN_OPS] + [T.bvcmp(op, a, b) for op in CMP_OPS] + \
            [T.bvun("bvneg", a), T.bvun("bvnot", a), T.bvexp(a, b)]
    vals = EDGE_256 + [(1 << 256) - 5, 3 << 254, 0x1234567890ABCDEF << 100, 7]
    assigns = [[x, y] for x in vals for y in vals]
    P, _, ver, got, models = gpu_eval_terms(engine, [T.BoolVal(True)], terms, assigns)
    for i, (x, y) in enumerate(assigns):
        want = evaluate_many(terms, OracleModel({"a": x, "b": y}))
        for t, w in zip(terms, want):
            assert got[i][t.id] == w, (t.op, hex(x), hex(y))


def test_narrow_widths(engine):
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
        P, _, ver, got, models = gpu_eval_terms(engine, [T.BoolVal(True)], terms, assigns)
        for i, (x, y) in enumerate(assigns):
            want = evaluate_many(terms, OracleModel({"a": x, "b": y}))
            for t, wv in zip(terms, want):
                assert got[i][t.id] == wv, (w, t.op, x, y)


def test_search_finds_verified_model_bectoken(engine):
    """BECToken batchOverflow (C3 shape): the GPU model satisfies every constraint
    under the oracle."""
    from test_host_boundary import _bec_constraints

    cs = _bec_constraints()
    roots = [c.raw for c in cs]
    res = search.search(engine, roots, seed=0x6D797468, max_candidates=1 << 26, timeout_s=60)
    assert res.index is not None, "no model found"
    ver, scalars, arrays, funcs, P = res.model
    assert ver == 1
    m = OracleModel(scalars, arrays, funcs)
    assert all(evaluate(r, m) == 1 for r in roots)


def test_search_deterministic_across_shards(engine):
    """The first hit is the global minimum index whatever the chunking (1/2/4 'GPUs')."""
    x = symbol_factory.BitVecSym("x", 256)
    y = symbol_factory.BitVecSym("y", 256)
    cs = [ULT(x, BVV(1 << 20, 256)), UGT(y, x), (x & BVV(0xFF, 256)) == 0x3C]
    roots = [c.raw for c in cs]
    P = ssa.flatten(roots)
    g = search.default_generator(P)
    blob = g.blob()
    prog = engine.load(P.to_bytes())
    gh = engine.load_gen(prog, blob)
    try:
        full, _ = engine.search(prog, gh, 99, 0, 1 << 20, early_exit=True)
        assert full is not None
        for shards in (2, 4):
            per = (1 << 20) // shards
            hits = [engine.search(prog, gh, 99, s * per, per, early_exit=True)[0] for s in range(shards)]
            hits = [h for h in hits if h is not None]
            assert min(hits) == full
        # no early exit: same first hit, and hit count equals the eval verdict count
        idx, nh = engine.search(prog, gh, 99, 0, 1 << 16, early_exit=False)
        ver, _ = engine.eval_generated(prog, gh, 99, 0, 1 << 16)
        assert nh == int(ver.sum())
        if nh:
            assert idx == int(np.flatnonzero(ver)[0])
    finally:
        engine.free_gen(gh)
        engine.free(prog)


def test_keccak_uf_sat_cases(engine):
    """tests/laser/keccak_tests.py sat verdicts: the UF side conditions of
    keccak_function_manager.py:121-149 are satisfiable and the GPU finds a model."""
    TOTAL_PARTS = 10 ** 40
    PART = (2 ** 256 - 1) // TOTAL_PARTS
    idx = TOTAL_PARTS - 34534
    lo, hi = idx * PART, idx * PART + PART
    f = Function("keccak256_256", 256, 256)
    inv = Function("keccak256_256-1", 256, 256)

    def cond(x):
        from mythril_amd.smt import ULE, URem

        return And(inv(f(x)) == x, ULE(BVV(lo, 256), f(x)), ULT(f(x), BVV(hi, 256)), URem(f(x), BVV(64, 256)) == 0)

    n1 = symbol_factory.BitVecSym("N1", 256)
    n2 = symbol_factory.BitVecSym("N2", 256)
    roots = [cond(n1).raw, cond(n2).raw, (f(n1) == f(n2)).raw]
    res = search.search(engine, roots, max_candidates=1 << 24, timeout_s=60)
    assert res.index is not None
    ver, scalars, arrays, funcs, P = res.model
    m = OracleModel(scalars, arrays, funcs)
    assert all(evaluate(r, m) == 1 for r in roots)
    assert scalars["N1"] == scalars["N2"]


def test_eval_dev_resident_inputs(engine):
    """The HBM-resident entry point used by bench.py agrees with mg_eval."""
    x = symbol_factory.BitVecSym("x", 256)
    y = symbol_factory.BitVecSym("y", 256)
    c = Not(BVMulNoOverflow(x, y, False))
    P = ssa.flatten([c.raw])
    n = 4096
    assigns = random_assignments(P, n, 5)
    soa = ssa.soa_from_assignments(P, assigns)
    prog = engine.load(P.to_bytes())
    try:
        ver_h, _ = engine.eval(prog, soa, n)
        d_soa = engine.dev_alloc(soa.nbytes)
        d_ver = engine.dev_alloc(n)
        engine.dev_upload(d_soa, soa)
        engine.eval_dev(prog, d_soa, n, d_ver)
        ver_d = np.zeros(n, dtype=np.uint8)
        engine.dev_download(ver_d, d_ver)
        engine.dev_free(d_soa)
        engine.dev_free(d_ver)
    finally:
        engine.free(prog)
    assert (ver_h == ver_d).all()
    for i in range(0, n, 97):
        assert ver_h[i] == evaluate(c.raw, OracleModel({"x": assigns[i][0], "y": assigns[i][1]}))


WORKLOAD_NAMES = ["token_transfer_underflow", "etherstore_reentrancy", "bectoken_batch_overflow",
                  "walletlibrary_kill", "sha3_keyed_mapping"]


@pytest.mark.parametrize("aux", [False, True])
@pytest.mark.parametrize("shaped", [False, True])
@pytest.mark.parametrize("name", WORKLOAD_NAMES, ids=workloads.test_id)
def test_workload_verdicts_match_c_restatement(engine, name, shaped, aux):
    """Every candidate verdict of the benchmark workloads (search-mode generator, broad
    or propagation-shaped; full evaluation) equals the C restatement's, and the search
    first hit/count agree."""
    from mythril_amd import workloads
    from oracle import cport

    roots = [c.raw for c in workloads.WORKLOADS[name]()]
    P = ssa.flatten(roots, aux_words=aux)
    blob = search.default_generator(P, roots=roots if shaped else None).blob()
    n, start, seed = 1 << 14, 12345, 0x6D797468
    prog = engine.load(P.to_bytes())
    gh = engine.load_gen(prog, blob)
    try:
        gver, _ = engine.eval_generated(prog, gh, seed, start, n)
        gfirst, ghits = engine.search(prog, gh, seed, start, n, early_exit=False)
    finally:
        engine.free_gen(gh)
        engine.free(prog)
    cfirst, chits, cver = cport.search(P.to_bytes(), blob, seed, start, n, threads=8, verdicts=True)
    assert (gver == cver).all(), int((gver != cver).sum())
    assert (gfirst, ghits) == (cfirst, chits)


@pytest.mark.parametrize("name", WORKLOAD_NAMES, ids=workloads.test_id)
def test_workload_models_verified(engine, name):
    """The GPU finds a model of each workload query and the oracle accepts it."""
    from mythril_amd import workloads

    roots = [c.raw for c in workloads.WORKLOADS[name]()]
    res = search.search(engine, roots, max_candidates=1 << 28, timeout_s=60)
    assert res.index is not None, name
    ver, scalars, arrays, funcs, P = res.model
    m = OracleModel(scalars, arrays, funcs)
    assert ver == 1 and all(evaluate(r, m) == 1 for r in roots)


def test_power_of_two_strength_reduction(engine):
    """udiv/urem/mul by a literal 2^k are lowered to extract/zext/concat; exact vs the oracle,
    in both the interpreter and the JIT kernels."""
    a = T.BitVecVar("a", 256)
    terms = []
    for k in (0, 1, 5, 31, 32, 33, 64, 200, 224, 255):
        c = T.BitVecVal(1 << k, 256)
        terms += [T.bvbin("bvudiv", a, c), T.bvbin("bvurem", a, c), T.bvbin("bvmul", a, c)]
    a8 = T.BitVecVar("a8", 8)
    terms += [T.bvbin(op, a8, T.BitVecVal(1 << k, 8)) for op in ("bvudiv", "bvurem", "bvmul") for k in (0, 3, 7)]
    rng = random.Random(11)
    assigns = [[rng.getrandbits(256), rng.getrandbits(8)] for _ in range(200)] + [[(1 << 256) - 1, 255], [0, 0]]
    P, _, ver, got, models = gpu_eval_terms(engine, [T.BoolVal(True)], terms, assigns)
    for i, (x, y) in enumerate(assigns):
        want = evaluate_many(terms, OracleModel({"a": x, "a8": y}))
        for t, w in zip(terms, want):
            assert got[i][t.id] == w, (t.op, T.to_sexpr(t.args[1]), hex(x))
    # the JIT path on the same program
    P2 = ssa.flatten([T.BoolVal(True)], extra=terms)
    P2.set_watch([P2.term_node[t.id] for t in terms])
    soa = ssa.soa_from_assignments(P2, assigns)
    prog = engine.load(P2.to_bytes())
    try:
        info = engine.info(prog)
        vi, wi = engine.eval(prog, soa, len(assigns), watch_words=info.watch_words)
        jit = engine.jit_compile(prog, 0)
        vj, wj = engine.jit_eval(jit, soa, len(assigns), watch_words=info.watch_words)
        engine.jit_free(jit)
    finally:
        engine.free(prog)
    assert (wi == wj).all()


@pytest.mark.parametrize("jit", [False, True, "o3"])
def test_division_operand_sizes(engine, jit):
    """udivrem8's paths (one-limb long division, quotient-bit loop with 2/4/8-limb
    remainders) under every mix of operand sizes within a wave: per-lane bit lengths of
    dividend and divisor from 0 to 256, a < b, a = b, b = 1, b = 0, signed edge values."""
    from helpers import gpu_eval_terms

    rng = random.Random(11)
    a = T.BitVecVar("a", 256)
    b = T.BitVecVar("b", 256)
    terms = [T.bvbin(op, a, b) for op in ["bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"]]

    def val(bits):
        return rng.getrandbits(bits) | (1 << (bits - 1)) if bits else 0

    assigns = []
    for _ in range(6 * 64):
        la, lb = rng.choice([0, 1, 2, 31, 32, 33, 64, 65, 96, 128, 129, 200, 255, 256]), \
            rng.choice([0, 1, 2, 3, 31, 32, 33, 63, 64, 65, 127, 128, 160, 255, 256])
        assigns.append([val(la), val(lb)])
    # waves with one-limb divisors only, and the edge pairs
    assigns += [[rng.getrandbits(256), rng.choice([1, 2, 3, 7, 10, 0xFFFFFFFF, 0])] for _ in range(128)]
    edges = [0, 1, 2, 3, (1 << 255), (1 << 255) - 1, (1 << 256) - 1, (1 << 256) - 2, 1 << 128, (1 << 32) - 1, 1 << 32]
    assigns += [[x, y] for x in edges for y in edges]
    # jit=True: the default watch-row kernel (the first tier's), "o3": the O3 kernel
    P, _, ver, got, models = gpu_eval_terms(engine, [T.BoolVal(True)], terms, assigns, jit=bool(jit), o3=jit == "o3")
    for i, (x, y) in enumerate(assigns):
        want = evaluate_many(terms, OracleModel({"a": x, "b": y}))
        for t, w in zip(terms, want):
            assert got[i][t.id] == w, (t.op, hex(x), hex(y))
