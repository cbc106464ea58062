"""The watch-row capture of a latency-bound interpreter search (one 64-index group per block,
engine.hip mg_search) returns the same model as the second-pass read-back (read_assignment)."""
import numpy as np
import pytest

from mythril_amd import native, search, workloads

pytestmark = pytest.mark.gpu

SEED = 0x6D797468


@pytest.mark.parametrize("name", ["suicide_kill", "token_transfer_underflow", "etherstore_reentrancy",
                                  "bectoken_batch_overflow", "walletlibrary_kill"], ids=workloads.test_id)
def test_capture_matches_readback(name):
    eng = native.Engine.get()
    roots = [c.raw for c in workloads.WORKLOADS[name]()]
    P, blob = search.prepare(roots)
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    try:
        ww = max(P.watch_words, 1)
        # capture: a small launch (every block sweeps one group); read-back: a launch far larger
        # than one group per block, starting at the same group, so it finds the same first hit
        a_cap = np.zeros(ww, dtype=np.uint32)
        a_rb = np.zeros(ww, dtype=np.uint32)
        start = 0
        for _ in range(64):
            idx, _ = eng.search(prog, gh, SEED, start, 1 << 12, early_exit=True, assign=a_cap)
            if idx is not None:
                break
            start += 1 << 12
        assert idx is not None, "no hit in the first 2^18 candidates"
        idx2, _ = eng.search(prog, gh, SEED, start, 1 << 24, early_exit=True, assign=a_rb)
        assert idx2 == idx
        assert np.array_equal(a_cap, a_rb)
    finally:
        eng.free_gen(gh)
        eng.free(prog)
