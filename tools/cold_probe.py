"""Where a cold easy query's time goes (GPU box): engine caches cleared before each query, then
search.search with its timing split, the first launch's kernel time from the engine's stats, and
a warm repeat.  python tools/cold_probe.py [workload] -> JSON lines"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from mythril_amd import native, search, ssa, workloads  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "token_transfer_underflow"
eng = native.Engine.get()
roots = [c.raw for c in workloads.WORKLOADS[w]()]
for trial in range(6):
    cold = trial % 2 == 0
    if cold:
        search.FLATTEN_CACHE = ssa.FlattenCache(aux_words=True)
        search._GEN_CACHE.clear()
        eng.cache_clear()
    eng.reset_stats()
    t = time.perf_counter()
    r = search.search(eng, roots, max_candidates=1 << 30, timeout_s=10)
    ms = (time.perf_counter() - t) * 1e3
    st = eng.stats()
    print(json.dumps({"trial": trial, "cold": cold, "ms": round(ms, 3), "timing": getattr(r, "timing", None),
                      "launches": st.launches, "kernel_ms_total": round(st.kernel_ms_total, 4),
                      "index": r.index, "engine": r.engine}), flush=True)
