"""Simulated LASER query stream through ``solver.get_model`` (the drop-in's hot call).

LASER asks ``get_model`` once per feasibility check as it walks a path: the constraint
list grows by one condition per JUMPI, and each branch point yields two sibling queries
(the condition and its negation, ``laser/ethereum/instructions.py`` jumpi_).  This
replays that shape over the C1-C4 workloads: for every prefix of a workload's constraint
list, the prefix itself (the taken branch) and the prefix with its last condition negated
(the sibling), plus one hard sibling per workload: the full path with a 64-bit needle on one
of its own 256-bit symbols (``Extract(63, 0, v * K) == C``, ~2^-64 per candidate), which no
budget can satisfy — it runs the whole slice, as LASER's infeasible branches do under z3.
Every query goes through ``solver.get_model`` with ``args.solver_timeout`` = the hook's
default 200 ms budget, so flattening (``FlattenCache``), generator, launches, the async
JIT compile and the model read-back are all inside the measured time.

Prints one JSON line per workload and a summary:
  budget_bound_rate   candidates / second over the queries that ran out of budget
  stream_rate         candidates / second over the whole stream

``--race-z3-ms D`` instead runs every query through the hook's race core (``plugin.race``, the
same code ``get_model`` runs inside Mythril) against a z3 stand-in that "solves" for D ms on its
worker thread and then answers unsat (there is no z3 on the box).  The GPU side is the real
search (``search_partitioned`` with the race's cancel event and launch cap).  Reported: for the
queries the stand-in answered (GPU misses), the hook's wall time beyond z3's own — the latency a
miss adds — and for the queries the GPU won, their wall time.
usage: python tools/stream_bench.py [--budget-ms 200] [--workloads a,b] [--race-z3-ms 50]
"""
import argparse
import json
import statistics
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from mythril_amd import search, solver, workloads  # noqa: E402
from mythril_amd.smt import BitVec, Extract, Not, symbol_factory  # noqa: E402
from mythril_amd.smt import terms as T  # noqa: E402

SHAPES = ["suicide_kill", "token_transfer_underflow", "etherstore_reentrancy", "bectoken_batch_overflow",
          "walletlibrary_kill"]


def stream_queries(name):
    """(label, constraints) in LASER order: prefixes, negated siblings, one infeasible sibling."""
    cs = list(workloads.WORKLOADS[name]())
    out = []
    for k in range(1, len(cs) + 1):
        out.append((f"prefix{k}", tuple(cs[:k])))
        if k >= 2:
            out.append((f"sibling{k}", tuple(cs[:k - 1]) + (Not(cs[k - 1]),)))
    v = next(t for t in T.postorder([c.raw for c in cs]) if t.op == "bvvar" and t.width == 256)
    k = symbol_factory.BitVecVal(0x9E3779B97F4A7C15F39CC0605CEDC835, 256)
    needle = Extract(63, 0, BitVec(v) * k) == symbol_factory.BitVecVal(0x0123456789ABCDEF, 64)
    out.append(("hard", tuple(cs) + (needle,)))
    return out


class StandInZ3:
    """The z3 side of the race on a box without z3: D ms of interruptible "solving", then unsat."""

    def __init__(self, delay_s: float):
        self.delay_s = delay_s
        self.stop = threading.Event()
        self.result = None
        self.seconds = 0.0

    def run(self):
        t0 = time.perf_counter()
        self.result = "unknown" if self.stop.wait(self.delay_s) else "unsat"
        self.seconds = time.perf_counter() - t0
        return self

    def interrupt(self):
        self.stop.set()


def run_race(names, budget_ms, z3_ms, quiet=False):
    """Every stream query through ``plugin.race`` (GPU search vs the z3 stand-in)."""
    from mythril_amd import native, plugin

    eng = native.Engine.get()
    rows = []
    for name in names:
        added, gpu_wall = [], []
        for label, q in stream_queries(name):
            roots = [c.raw for c in q]
            z3j = StandInZ3(z3_ms / 1e3)
            t = time.perf_counter()
            winner, out = plugin.race(
                lambda cancel: search.search_partitioned(eng, roots, timeout_s=budget_ms / 1e3,
                                                         max_candidates=1 << 40, cancel=cancel,
                                                         max_launch_s=plugin.RACE_LAUNCH_S),
                z3j, lambda res: res if res is not None and res.index is not None else None)
            dt = time.perf_counter() - t
            if winner == "gpu":
                gpu_wall.append(dt * 1e3)
            else:
                added.append((dt - out.seconds) * 1e3)
        row = {"workload": name, "race_z3_standin_ms": z3_ms, "gpu_won": len(gpu_wall), "z3_won": len(added),
               "added_ms_per_miss_median": round(statistics.median(added), 3) if added else None,
               "added_ms_per_miss_max": round(max(added), 3) if added else None,
               "gpu_won_wall_ms_median": round(statistics.median(gpu_wall), 3) if gpu_wall else None}
        rows.append(row)
        if not quiet:
            print(json.dumps(row), flush=True)
    return rows


def run(names, budget_ms, verbose=False, quiet=False):
    solver.args.solver_timeout = budget_ms
    st = solver.SolverStatistics()
    rows = []
    for name in names:
        qs = stream_queries(name)
        solver.get_model.cache_clear()
        t_all = time.perf_counter()
        cand_all = 0
        bound_t = bound_c = 0.0
        engines = {}
        n_sat = 0
        for label, q in qs:
            c0 = st.candidates
            t = time.perf_counter()
            try:
                solver.get_model(q, enforce_execution_time=False)
                n_sat += 1
            except solver.UnsatError:
                pass
            dt = time.perf_counter() - t
            dc = st.candidates - c0
            cand_all += dc
            if dt >= 0.9 * budget_ms / 1e3:
                bound_t += dt
                bound_c += dc
            eng = getattr(search, "LAST_ENGINE", None)
            if eng:
                engines[eng] = engines.get(eng, 0) + 1
            if verbose:
                r = search.LAST_RESULT
                print(json.dumps({"q": label, "ms": round(dt * 1e3, 2), "candidates": int(dc), "engine": eng,
                                  "timing": {k: round(v, 2) for k, v in (r.timing if r else {}).items()}}),
                      flush=True)
        total = time.perf_counter() - t_all
        row = {"workload": name, "queries": len(qs), "sat": n_sat, "budget_ms": budget_ms,
               "stream_s": round(total, 4), "candidates": int(cand_all),
               "stream_rate": cand_all / total if total else 0.0,
               "budget_bound_queries_s": round(bound_t, 4),
               "budget_bound_rate": bound_c / bound_t if bound_t else None, "engines": engines}
        rows.append(row)
        if not quiet:
            print(json.dumps(row), flush=True)
    bt = sum(r["budget_bound_queries_s"] for r in rows)
    bc = sum((r["budget_bound_rate"] or 0) * r["budget_bound_queries_s"] for r in rows)
    summary = {"summary": True, "budget_ms": budget_ms, "workloads": len(rows),
               "budget_bound_rate": bc / bt if bt else None,
               "stream_rate": sum(r["candidates"] for r in rows) / sum(r["stream_s"] for r in rows),
               "jit_compile_s_avg": search.JIT_COMPILE_S[0]}
    if not quiet:
        print(json.dumps(summary), flush=True)
    return rows, summary


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget-ms", type=float, default=200.0)
    ap.add_argument("--workloads", default=",".join(SHAPES))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--race-z3-ms", type=float, default=None)
    a = ap.parse_args()
    names = [w for w in a.workloads.split(",") if w]
    if a.race_z3_ms is not None:
        run_race(names, a.budget_ms, a.race_z3_ms)
    else:
        run(names, a.budget_ms, a.verbose)


if __name__ == "__main__":
    main()
