"""Per-candidate parity sweep at random 63-bit index windows, every BASELINE config.

For each workload (test id = the BASELINE.json config it stands for), two random seeds and four
random unaligned windows of 2,048 candidates each, the verdict of every candidate from

* the compiled search kernel's body (``mgj_gen`` via ``mg_jit_verdicts``), and
* the interpreter in generator mode (``k_run`` via ``mg_eval_generated``)

must equal the C port's (``oracle/bveval.c``, ``cport.search(verdicts=True)``) on the same GEN3
candidate stream.  Two of the four windows start with bit 31 of the low index word set: the 64-bit
group base bug found in round 2 (a sign-extended low word) lived exactly there.  Then the search
entry points must report the C port's first hit and hit count on each window.

Reference anchor: the candidate verdict is ``Model.eval(And(constraints), model_completion=True)``
(``mythril/laser/smt/model.py:45-59``) of the query ``get_model`` receives
(``mythril/support/model.py:15-49``); the workloads' term shapes follow SURVEY.md §8(d) C1-C5.
"""
import random
import zlib

import numpy as np
import pytest

from mythril_amd import search, workloads

pytestmark = pytest.mark.gpu

N = 2048
SEEDS = 2
WINDOWS = 4


def _windows(rng):
    out = []
    for w in range(WINDOWS):
        start = rng.getrandbits(63)
        if w < 2:  # low word with bit 31 set, unaligned inside its 64-index group
            start = (start & ~0xFFFFFFFF) | 0x80000000 | rng.getrandbits(31)
        start |= 1  # never group-aligned
        out.append(start)
    return out


@pytest.mark.parametrize("name", sorted(workloads.WORKLOADS), ids=workloads.test_id)
def test_sweep_random_windows(engine, name):
    _sweep(engine, name, [c.raw for c in workloads.WORKLOADS[name]()])


def test_sweep_literal_tail_keys(engine):
    """Keys Concat(key, literal slot) compared through EQ, ITE and keccak sites: the interpreter
    runs them narrowed to the key halves (program.cpp: narrow_literal_tails), mixed tails included."""
    from tests.helpers import literal_tail_query

    _sweep(engine, "literal_tail_keys", [c.raw for c in literal_tail_query()])


def _sweep(engine, name, roots):
    from oracle import cport

    rng = random.Random(zlib.crc32(name.encode()) ^ 0x6D797468)
    P, blob = search.prepare(roots)
    pb = P.to_bytes()
    prog = engine.load(pb)
    gh = engine.load_gen(prog, blob)
    jh = engine.jit_compile(prog, gh, gen_verdicts=True)
    total = hits = 0
    try:
        for _ in range(SEEDS):
            seed = rng.getrandbits(32)
            for start in _windows(rng):
                cf, ch, want = cport.search(pb, blob, seed, start, N, threads=16, verdicts=True)
                vj = engine.jit_verdicts(jh, seed, start, N)
                vi, _ = engine.eval_generated(prog, gh, seed, start, N)
                bj = np.nonzero(vj != want)[0]
                bi = np.nonzero(vi != want)[0]
                assert bj.size == 0, f"JIT: {bj.size} mismatches, first at index {start + int(bj[0])} seed {seed}"
                assert bi.size == 0, f"interp: {bi.size} mismatches, first at index {start + int(bi[0])} seed {seed}"
                # the search entry points agree on the first hit and count of the window
                assert engine.jit_search(jh, seed, start, N, early_exit=False) == (cf, ch)
                assert engine.search(prog, gh, seed, start, N, early_exit=False) == (cf, ch)
                total += N
                hits += int(want.sum())
    finally:
        engine.jit_free(jh)
        engine.free_gen(gh)
        engine.free(prog)
    assert total == SEEDS * WINDOWS * N
