"""Fixed per-call latency of the search entry points (GPU box): the time-to-first-model floor.
usage: python tools/latency_probe.py [workload]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from mythril_amd import native, search, workloads  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "token_transfer_underflow"
eng = native.Engine.get()
roots = [c.raw for c in workloads.WORKLOADS[w]()]
P, blob = search.prepare(roots)
out = {}


def t(label, fn, reps=50):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    out[label] = round(1e6 * float(np.median(ts)), 1)


t("prepare_us (caches warm)", lambda: search.prepare(roots))
prog = eng.load(P.to_bytes())
gh = eng.load_gen(prog, blob)
t("load_us", lambda: eng.free(eng.load(P.to_bytes())))
t("load_gen_us", lambda: eng.free_gen(eng.load_gen(prog, blob)))
assign = np.zeros(max(P.watch_words, 1), dtype=np.uint32)
for n in (64, 1 << 12, 1 << 16, 1 << 20):
    t(f"search_{n}_us", lambda n=n: eng.search(prog, gh, 7, 1 << 40, n, early_exit=True))
for n in (64, 1 << 16):
    eng.search(prog, gh, 7, 1 << 40, n, early_exit=True)
    out[f"search_{n}_kernel_us"] = round(1e3 * eng.stats().last_kernel_ms, 1)
# a one-constraint program: the fixed cost of a search call (launch, hit-buffer copies, sync)
from mythril_amd.smt import symbol_factory as _sf  # noqa: E402
_x = _sf.BitVecSym("probe_x", 8)
P1, blob1 = search.prepare([(_x == _sf.BitVecVal(5, 8)).raw])
prog1 = eng.load(P1.to_bytes())
gh1 = eng.load_gen(prog1, blob1)
t("trivial_search_64_us", lambda: eng.search(prog1, gh1, 7, 1 << 40, 64, early_exit=True))
eng.search(prog1, gh1, 7, 1 << 40, 64, early_exit=True)
out["trivial_search_64_kernel_us"] = round(1e3 * eng.stats().last_kernel_ms, 1)
t("search_hit_with_assign_us", lambda: eng.search(prog, gh, 7, 0, 1 << 16, early_exit=True, assign=assign))
t("keccak_1_us", lambda: eng.keccak256([b"abc"]))
t("search_py_total_us", lambda: search.search(eng, roots, timeout_s=10, jit="never"))
r = search.search(eng, roots, timeout_s=10, jit="never")
out["search_py_timing"] = {k: round(v * 1e3, 1) for k, v in r.timing.items()}
print(json.dumps(out))
