"""Multi-device search inside the shim (no torch.distributed): mg_init with several devices
splits every mg_search / mg_jit_search over them (mg_split_range) and reduces on the host.
The box has one MI355X, so MYTHGPU_VIRTUAL_DEVICES=k opens k logical devices on it (own
streams, buffers, mirrored handles, per-device JIT module loads) — the same split,
mirroring and reduction code as k physical GPUs.  The first hit and hit count must equal
the single-device engine's on every workload, interpreter and JIT."""
import os

import pytest

from mythril_amd import search, workloads

# MYTHGPU_TIMING_ASSERTS=1 (tools/timing_checks.sh) turns the wall-clock bounds into assertions; the
# parity run (pytest -m gpu) only prints them, so a slow or noisy box cannot fail it on timing
TIMING = os.environ.get("MYTHGPU_TIMING_ASSERTS") == "1"
pytestmark = pytest.mark.gpu

NAMES = ["token_transfer_underflow", "bectoken_batch_overflow", "walletlibrary_kill", "sha3_keyed_mapping"]


def _run(engine, P, blob, windows, jit):
    prog = engine.load(P.to_bytes())
    gh = engine.load_gen(prog, blob)
    out = []
    try:
        jh = engine.jit_compile(prog, gh) if jit else None
        for (s, n, early) in windows:
            if jh is not None:
                r = engine.jit_search(jh, 7, s, n, early_exit=early)
            else:
                r = engine.search(prog, gh, 7, s, n, early_exit=early)
            # with early exit the hit count depends on when waves see the first hit
            out.append(r[0] if early else r)
        if jh is not None:
            engine.jit_free(jh)
    finally:
        engine.free_gen(gh)
        engine.free(prog)
    return out


def test_full_mask_and_virtual_devices_same_hits(engine):
    windows = [(0, 1 << 22, True), (0, 1 << 22, False), (12345, (1 << 21) + 77, False), (1 << 33, 1 << 20, True),
               (5, 3, False)]
    cases = []
    for name in NAMES:
        roots = [c.raw for c in workloads.WORKLOADS[name]()]
        P, blob = search.prepare(roots)
        cases.append((name, P, blob))
    single = {(name, jit): _run(engine, P, blob, windows, jit) for name, P, blob in cases for jit in (False, True)}
    old_mask = engine.mask
    try:
        # every device of the box (one MI355X here): the multi-device code path with one slice
        engine.reinit(0xFFFFFFFF)
        for name, P, blob in cases:
            for jit in (False, True):
                assert _run(engine, P, blob, windows, jit) == single[(name, jit)], (name, jit, "full mask")
        # four logical devices on it: four slices per call, host min / sum — with the default
        # split threshold (only launches of >= 2^20 candidates per device are split) and with
        # every launch split (MYTHGPU_SPLIT_MIN=64)
        os.environ["MYTHGPU_VIRTUAL_DEVICES"] = "4"
        engine.reinit(1 << engine.device)
        assert engine.n_devices == 4
        for split_min in (None, "64"):
            if split_min:
                os.environ["MYTHGPU_SPLIT_MIN"] = split_min
            for name, P, blob in cases:
                for jit in (False, True):
                    assert _run(engine, P, blob, windows, jit) == single[(name, jit)], (name, jit, "4 devices",
                                                                                          split_min)
            os.environ.pop("MYTHGPU_SPLIT_MIN", None)
        # the search loop and the model read-back on top of it
        roots = [c.raw for c in workloads.WORKLOADS["token_transfer_underflow"]()]
        r = search.search(engine, roots, timeout_s=10, jit="never")
        assert r.index is not None and r.model[0] == 1
    finally:
        os.environ.pop("MYTHGPU_VIRTUAL_DEVICES", None)
        os.environ.pop("MYTHGPU_SPLIT_MIN", None)
        engine.reinit(old_mask)
    assert engine.n_devices == 1


def _ttfm(engine, roots, reps=9):
    import statistics
    import time

    search.search(engine, roots, timeout_s=10)  # warm: caches, capture buffers, code
    out, idx = [], set()
    for _ in range(reps):
        t = time.perf_counter()
        r = search.search(engine, roots, timeout_s=10)
        out.append(time.perf_counter() - t)
        idx.add(r.index)
    return statistics.median(out), idx


def test_time_to_first_model_at_four_devices(engine):
    """An easy query's first launch (2^12 candidates) stays on device 0 with the model capture at
    N > 1, so time to first model does not regress with the device count (C2 within 10 %, same hit)."""
    roots = [c.raw for c in workloads.WORKLOADS["token_transfer_underflow"]()]
    t1, i1 = _ttfm(engine, roots)
    old_mask = engine.mask
    try:
        os.environ["MYTHGPU_VIRTUAL_DEVICES"] = "4"
        engine.reinit(1 << engine.device)
        assert engine.n_devices == 4
        t4, i4 = _ttfm(engine, roots)
    finally:
        os.environ.pop("MYTHGPU_VIRTUAL_DEVICES", None)
        engine.reinit(old_mask)
    assert i1 == i4 and len(i1) == 1
    print(f"time to first model: 1 device {t1 * 1e3:.3f} ms, 4 devices {t4 * 1e3:.3f} ms")
    if TIMING:  # wall-clock bound: tools/timing_checks.sh, not the parity run
        assert t4 <= 1.10 * t1 + 50e-6, (t1, t4)


def test_multidevice_stops_at_first_hit(engine):
    """A mid-range needle (~2^-20) whose first hit lies in slice 0 of a 2^24 launch split over four
    devices: the wave that finds it lowers the hit words of the devices above (engine.hip peer
    line), so their waves stop at the next group instead of sweeping their whole slice.  Same index
    as one device, on the O3 kernel, the first tier and the interpreter; the split launch's time
    stays within 1.1x of one device's plus the three extra launches (25 us each)."""
    import statistics
    import time

    from mythril_amd.smt import Extract, symbol_factory

    x = symbol_factory.BitVecSym("md_needle_x", 256)
    k = symbol_factory.BitVecVal(0x9E3779B97F4A7C15F39CC0605CEDC835, 256)
    roots = [(Extract(19, 0, x * k) == symbol_factory.BitVecVal(0x5A5A5, 20)).raw]
    P, blob = search.prepare(roots)
    n = 1 << 24

    def kernels():
        prog = engine.load(P.to_bytes())
        gh = engine.load_gen(prog, blob)
        return prog, gh, {"o3": engine.jit_compile(prog, gh), "asm": engine.jit_compile(prog, gh, asm=True)}

    def timed(fn, reps=15):
        fn()
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            r = fn()
            ts.append(time.perf_counter() - t)
        return statistics.median(ts), r

    prog, gh, ks = kernels()
    try:
        seed = next(s for s in range(200)
                    if (1 << 20) <= (engine.jit_search(ks["o3"], s, 0, n, early_exit=True)[0] or n) < (1 << 22))
        one = {name: timed(lambda j=j: engine.jit_search(j, seed, 0, n, early_exit=True)[0]) for name, j in ks.items()}
        one["interp"] = timed(lambda: engine.search(prog, gh, seed, 0, n, early_exit=True)[0], reps=5)
    finally:
        for j in ks.values():
            engine.jit_free(j)
        engine.free_gen(gh)
        engine.free(prog)
    old_mask = engine.mask
    try:
        os.environ["MYTHGPU_VIRTUAL_DEVICES"] = "4"
        engine.reinit(1 << engine.device)
        assert engine.n_devices == 4
        prog, gh, ks = kernels()
        try:
            four = {name: timed(lambda j=j: engine.jit_search(j, seed, 0, n, early_exit=True)[0])
                    for name, j in ks.items()}
            four["interp"] = timed(lambda: engine.search(prog, gh, seed, 0, n, early_exit=True)[0], reps=5)
        finally:
            for j in ks.values():
                engine.jit_free(j)
            engine.free_gen(gh)
            engine.free(prog)
    finally:
        os.environ.pop("MYTHGPU_VIRTUAL_DEVICES", None)
        engine.reinit(old_mask)
    for name in one:
        (t1, i1), (t4, i4) = one[name], four[name]
        assert i1 == i4 and i1 < (1 << 22), (name, i1, i4)
        print(f"{name}: 1 device {t1 * 1e3:.3f} ms, 4 devices {t4 * 1e3:.3f} ms")
        if TIMING and name != "interp":  # wall-clock bound: tools/timing_checks.sh, not the parity run
            assert t4 <= 1.10 * t1 + 3 * 25e-6, (name, t1, t4)
