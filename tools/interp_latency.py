"""Single-wave latency of the generic interpreter (k_run): the time-to-first-model floor.
One 64-candidate launch = one wave on one CU running the program once, caches as a query meets
them.  For each op kind, chained programs of 16 and 96 ops (tools/interp_micro.py's chains):
microseconds per interpreted instruction for one wave; then the workloads' own search and
capture programs.  GPU box:  python tools/interp_latency.py  -> one JSON line per row."""
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import numpy as np  # noqa: E402

from interp_micro import chain  # noqa: E402
from mythril_amd import native, search, workloads  # noqa: E402

eng = native.Engine.get()


def one_wave_us(prog, gh, reps=21, start=1 << 40, assign=None):
    ts = []
    for r in range(reps):
        eng.search(prog, gh, 7 + r, start, 64, early_exit=False, assign=assign)
        ts.append(eng.stats().last_kernel_ms * 1e3)
    return statistics.median(ts[1:])


for kind in ["add256", "xor256", "ult256", "eq256", "ite256", "add8", "extract", "coord256"]:
    row = {"kind": kind}
    for n in (16, 96):
        P, blob = search.prepare(chain(kind, n))
        prog = eng.load(P.to_bytes())
        gh = eng.load_gen(prog, blob)
        row[f"n{n}"] = {"instrs": eng.gen_info(gh).n_instrs, "us": one_wave_us(prog, gh)}
        eng.free_gen(gh)
        eng.free(prog)
    d = row["n96"]["instrs"] - row["n16"]["instrs"]
    row["us_per_instr_one_wave"] = (row["n96"]["us"] - row["n16"]["us"]) / max(d, 1)
    print(json.dumps(row), flush=True)

for w in ["suicide_kill", "token_transfer_underflow", "bectoken_batch_overflow", "walletlibrary_kill"]:
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[w]()])
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    assign = np.zeros(max(P.watch_words, 1), dtype=np.uint32)
    row = {"workload": w, "search_instrs": eng.gen_info(gh).n_instrs,
           "search_us": one_wave_us(prog, gh), "capture_us": one_wave_us(prog, gh, start=0, assign=assign)}
    print(json.dumps(row), flush=True)
    eng.free_gen(gh)
    eng.free(prog)
