"""``mg_jit_search_many`` (independent searches of one kernel launched back to back over four
streams, one wait): every launch's first hit and hit count equal one ``mg_jit_search`` call's, for
the O3 kernel and the first tier, with and without early exit, on ragged launch sizes (empty,
unaligned, one group, more launches than one batch holds).

Reference anchor: each launch answers the query ``get_model`` receives
(``mythril/support/model.py:15-49``) over its own candidate window."""
import random

import pytest

from mythril_amd import search, workloads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("asm", [False, True])
@pytest.mark.parametrize("name", ["token_transfer_underflow", "etherstore_reentrancy"])
def test_search_many_equals_single_calls(engine, name, asm):
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
    prog = engine.load(P.to_bytes())
    gh = engine.load_gen(prog, blob)
    j = engine.jit_compile(prog, gh, asm=asm)
    rng = random.Random(11)
    try:
        n = 70  # more than one batch of 64 slots
        seeds = [rng.getrandbits(32) for _ in range(n)]
        starts = [0 if q % 3 == 0 else rng.getrandbits(40) | 1 for q in range(n)]
        counts = [[0, 1, 63, 64, 1000, 1 << 16, (1 << 20) + 17][q % 7] for q in range(n)]
        for early in (False, True):
            got = engine.jit_search_many(j, seeds, starts, counts, early_exit=early)
            for q in range(n):
                want = engine.jit_search(j, seeds[q], starts[q], counts[q], early_exit=early) if counts[q] else (None, 0)
                if early:
                    assert got[q][0] == want[0], (q, got[q], want)
                else:
                    assert got[q] == want, (q, got[q], want)
    finally:
        engine.jit_free(j)
        engine.free_gen(gh)
        engine.free(prog)


def test_search_many_over_virtual_devices(engine):
    """Four logical devices (MYTHGPU_VIRTUAL_DEVICES): launches big enough to split go through
    mg_jit_search one after the other (every device's slice, host min / sum), small ones through the
    batch on the primary device; both give one mg_jit_search's answers."""
    import os

    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS["token_transfer_underflow"]()])
    old_mask = engine.mask
    seeds, starts, counts = [3, 4, 5], [0, 1 << 33, 77], [1 << 22, 1 << 21, 4096]
    try:
        prog = engine.load(P.to_bytes())
        gh = engine.load_gen(prog, blob)
        j = engine.jit_compile(prog, gh)
        want = [engine.jit_search(j, s, a, c, early_exit=False) for s, a, c in zip(seeds, starts, counts)]
        engine.jit_free(j)
        engine.free_gen(gh)
        engine.free(prog)
        os.environ["MYTHGPU_VIRTUAL_DEVICES"] = "4"
        engine.reinit(1 << engine.device)
        assert engine.n_devices == 4
        prog = engine.load(P.to_bytes())
        gh = engine.load_gen(prog, blob)
        j = engine.jit_compile(prog, gh)
        try:
            assert engine.jit_search_many(j, seeds, starts, counts) == want
            assert engine.jit_search_many(j, seeds[2:], starts[2:], counts[2:]) == want[2:]
        finally:
            engine.jit_free(j)
            engine.free_gen(gh)
            engine.free(prog)
    finally:
        os.environ.pop("MYTHGPU_VIRTUAL_DEVICES", None)
        engine.reinit(old_mask)
    assert engine.n_devices == 1
