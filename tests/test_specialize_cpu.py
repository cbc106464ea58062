"""Specialisation keeps every verdict (CPU, no GPU).

A search does not run the program it was given: ``program.cpp: specialize_program`` first
folds every comparison the generator's value ranges, known bits and value sets decide, aliases
ITEs/ORs/ANDs on decided conditions, drops decided asserts and dead code.  Both GPU kernels
(the interpreter and the JIT) run that specialised program, so a wrong fold would change
verdicts on the GPU without any kernel bug.  Here the specialised program
(``mg_program_specialized``) is evaluated by the oracle's plain-Python evaluator of device ops
(``oracle/kops.py``) on exactly the candidates the generator draws (``bv_gen_soa`` in
``oracle/bveval.c``), and every verdict must equal the C port's on the *unspecialised* program.
The eval-mode specialisation (literal facts only) is checked the same way on random
assignments.

Reference anchor: a candidate's verdict is ``Model.eval(And(constraints), model_completion=True)``
(``mythril/laser/smt/model.py:45-59``); workloads follow SURVEY.md §8(d) C1-C5.
"""
import random
import zlib

import numpy as np
import pytest

from mythril_amd import native, search, ssa, workloads
from oracle import cport, kops
from tests.helpers import random_assignments

N = 384


def _coord_words(P):
    return sum(ssa.limbs(c.width) for c in P.coords)


@pytest.mark.parametrize("interp", [False, True], ids=["jit", "interp"])
@pytest.mark.parametrize("keep_watch", [False, True], ids=["search", "watch"])
@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS), ids=workloads.test_id)
def test_specialised_search_program_keeps_verdicts(name, keep_watch, interp):
    """``interp``: the interpreter's program (literal-tail keys narrowed), else the compiled kernel's."""
    rng = random.Random(zlib.crc32(name.encode()) ^ 0x5BEC)
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
    pb = P.to_bytes()
    spec = native.specialized_program(pb, blob, keep_watch=keep_watch, interp=interp)
    widths = [c.width for c in P.coords]
    n = N if name != "sha3_keyed_mapping" else 96
    for start in (0, rng.getrandbits(63) | 1):
        seed = rng.getrandbits(32)
        soa = cport.gen_soa(pb, blob, seed, start, n, _coord_words(P))
        want = cport.search(pb, blob, seed, start, n, threads=4, verdicts=True)[2]
        got = kops.verdicts(spec, soa, widths, n)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, f"{name}: specialised verdict differs at index {start + int(bad[0])} (seed {seed})"


@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS), ids=workloads.test_id)
def test_specialised_eval_program_keeps_verdicts(name):
    P = ssa.flatten([c.raw for c in workloads.WORKLOADS[name]()])
    pb = P.to_bytes()
    spec = native.specialized_program(pb, None)
    n = 128 if name != "sha3_keyed_mapping" else 48
    soa = ssa.soa_from_assignments(P, random_assignments(P, n, seed=zlib.crc32(name.encode())))
    want = cport.eval_soa(pb, soa, n)
    got = kops.verdicts(spec, soa, [c.width for c in P.coords], n)
    assert np.array_equal(got, want)


def test_specialisation_folds_actor_membership():
    """LASER pins every transaction's caller to the actors (``Or(caller == a, ...)``,
    ``mythril/laser/ethereum/transaction/symbolic.py``); with the sender drawn from that same
    set the disjunction is true for every candidate, so no instruction of it survives."""
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS["token_transfer_underflow"]()])
    senders = {c.index for c in P.coords if c.name.startswith("sender_")}
    assert senders

    def sender_eqs(spec):
        vids = {int(r[2]) for r in spec["code"] if int(r[0]) == kops.K_COORD and int(r[6]) in senders}
        return sum(1 for r in spec["code"] if int(r[0]) == kops.K_EQ and (int(r[3]) in vids or int(r[4]) in vids))

    assert sender_eqs(native.specialized_program(P.to_bytes(), None)) >= 6  # 3 actors x 2 transactions
    assert sender_eqs(native.specialized_program(P.to_bytes(), blob)) == 0


def _tiny_queries():
    from mythril_amd.smt import ULT, symbol_factory

    x = symbol_factory.BitVecSym("tiny_x", 8)
    y = symbol_factory.BitVecSym("tiny_y", 256)
    return {
        "one_narrow_constraint": [(x == symbol_factory.BitVecVal(5, 8)).raw],
        "one_wide_compare": [ULT(y, symbol_factory.BitVecVal(1000, 256)).raw],
    }


@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS) + sorted(_tiny_queries()))
def test_jit_kernels_compile_on_host(name):
    """Every kernel the JIT emits for a query compiles for gfx950 on the host (comgr in the
    helper process, no GPU): the search kernel of each workload, and of queries with no MIXED
    coordinate (no choice words), whose emission paths differ."""
    roots = _tiny_queries()[name] if name in _tiny_queries() else [c.raw for c in workloads.WORKLOADS[name]()]
    P, blob = search.prepare(roots)
    src = native.jit_source(P.to_bytes(), blob, compile=True)
    assert "mgj_search" in src


def test_literal_tail_keys_are_narrowed():
    """Mapping keys ``Concat(key, slot)`` with a literal slot (LASER's storage addressing through
    ``keccak(Concat(key, slot))``): comparisons of such keys (EQ, ITE arms, LOOKUP sites) run on the
    key halves (``program.cpp: narrow_literal_tails``), and the verdicts stay those of the C port on
    the unspecialised program — also where the keys carry different literal tails (they never
    compare equal, and the wide values stay)."""
    from tests.helpers import literal_tail_query

    cs = literal_tail_query()
    P, blob = search.prepare([c.raw for c in cs])
    pb = P.to_bytes()
    spec = native.specialized_program(pb, blob, interp=True)
    eq512 = [r for r in spec["code"] if int(r[0]) == kops.K_EQ and int(r[7]) == 512]
    assert not eq512, "a comparison of literal-tail keys was not narrowed"
    wide = native.specialized_program(pb, blob)  # the compiled kernel keeps the wide program
    assert [r for r in wide["code"] if int(r[0]) == kops.K_EQ and int(r[7]) == 512]
    rng = random.Random(0x7A11)
    for start in (0, rng.getrandbits(63) | 1):
        seed = rng.getrandbits(32)
        soa = cport.gen_soa(pb, blob, seed, start, N, _coord_words(P))
        want = cport.search(pb, blob, seed, start, N, threads=4, verdicts=True)[2]
        for prog in (spec, wide):
            got = kops.verdicts(prog, soa, [c.width for c in P.coords], N)
            assert np.array_equal(got, want)


@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS))
def test_asm_tier_assembles_on_host(name):
    """The JIT's first tier (jit_asm.cpp) for every workload (C5's Keccak, EXP and SDIV included since
    round 5): the emitted gfx950 assembly (mgj_search + mgj_gen) assembles and links through comgr on
    the host."""
    roots = [c.raw for c in workloads.WORKLOADS[name]()]
    P, blob = search.prepare(roots)
    src = native.jit_asm(P.to_bytes(), blob, compile=True)
    assert src.startswith("; mythgpu-asm") and "mgj_search:" in src and "mgj_gen:" in src
    # results leave through vector memory only: the only scalar-memory instructions are the
    # kernel-argument loads
    smem = [ln.split()[0] for ln in src.splitlines() if ln.strip().startswith("s_") and ("[0:1]" in ln)]
    assert set(smem) <= {"s_load_dwordx2", "s_load_dwordx8", "s_load_dwordx4", "s_load_dword"}


def test_asm_tier_random_programs_assemble_on_host():
    """Random programs over the tier's operators (tests/test_gpu_asm.py) emit and assemble on the host."""
    from tests.test_gpu_asm import _random_program

    for seed in range(24):
        P, blob = search.prepare(_random_program(1000 + seed, full=bool(seed & 1)))
        native.jit_asm(P.to_bytes(), blob, compile=True)


@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS))
def test_asm_eval_workloads_assemble_on_host(name):
    """The first tier's eval kernel of every workload inside the tier, verdicts only and with the
    model watch rows, row-major and tiled SoA: emits (the occupancy-sized row queue tries several
    depths, abandoning a kernel that runs out of registers midway) and assembles.  An abandoned
    kernel's cached compare differences once leaked into the next attempt (C4: VGPR released twice)."""
    P, _ = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
    prev = P.watch
    try:
        for watch in (False, True):
            P.set_watch(prev if watch else [])
            for tiled in (False, True):
                src = native.jit_asm(P.to_bytes(), None, compile=True, tiled=tiled)
                assert "mgj_eval:" in src
    finally:
        P.set_watch(prev)


def test_asm_eval_with_watch_rows_assembles_on_host():
    """The first tier's eval kernel (mgj_eval) with watch rows, as ``gpu_eval_terms`` builds it (24
    watched terms + the model read-back rows): emits and assembles for every random program; a value
    read last by its watch store is released (an earlier build leaked its registers and refused)."""
    from mythril_amd import ssa
    from mythril_amd.search import model_watch
    from mythril_amd.smt import terms as T
    from tests.test_gpu_asm import _random_program

    for seed in range(16):
        roots = _random_program(3000 + seed, full=bool(seed & 1))
        watch = [t for t in T.postorder(roots) if t.sort[0] == "bv"][:24]
        P = ssa.flatten(list(roots), extra=list(watch))
        me, _ = model_watch(P)
        P.set_watch([P.term_node[t.id] for t in watch] + me)
        src = native.jit_asm(P.to_bytes(), None, compile=True)
        assert "mgj_eval:" in src


def test_lookup_compare_pushdown_fires_and_keeps_verdicts():
    """``program.cpp: push_eq_into_lookup`` (the compiled kernels' program only): LASER's keccak
    bookkeeping asserts ``EQ(LOOKUP(k; (k_q, v_q)...; x), x)`` once per hashed site, which becomes a
    width-1 LOOKUP over the priors' compares.  C2 and C4 carry that shape: their compiled program has
    width-1 LOOKUPs and fewer wide ones than the interpreter's (which keeps the original form), and
    on C2 the interpreter's has none of width 1.  Verdicts against the C port: the workload tests
    above (``jit``)."""
    K_LOOKUP = 30
    for name in ("token_transfer_underflow", "walletlibrary_kill"):
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        jit = native.specialized_program(P.to_bytes(), blob)["code"]
        itp = native.specialized_program(P.to_bytes(), blob, interp=True)["code"]
        narrow = lambda code: int(np.sum((code[:, 0] == K_LOOKUP) & (code[:, 1] == 1)))
        wide = lambda code: int(np.sum((code[:, 0] == K_LOOKUP) & (code[:, 1] > 1)))
        assert narrow(jit) > 0, name
        assert wide(jit) < wide(itp), name
        if name == "token_transfer_underflow":
            assert narrow(itp) == 0


@pytest.mark.parametrize("seed", range(12))
def test_rewritten_random_programs_keep_verdicts(seed):
    """Random programs over the tier's operators (``tests/test_gpu_asm.py``: LOOKUP sites, ITE chains,
    EQs), specialised for their generator: the compiled kernels' program — with the compare
    pushdown and the guarded-lookup pruning — gives the C port's verdicts on the unspecialised one."""
    from tests.test_gpu_asm import _random_program

    P, blob = search.prepare(_random_program(7000 + seed))
    pb = P.to_bytes()
    spec = native.specialized_program(pb, blob)
    widths = [c.width for c in P.coords]
    soa = cport.gen_soa(pb, blob, 11 + seed, 0, N, _coord_words(P))
    want = cport.search(pb, blob, 11 + seed, 0, N, threads=4, verdicts=True)[2]
    got = kops.verdicts(spec, soa, widths, N)
    assert np.array_equal(got, want)
