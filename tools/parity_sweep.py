"""Per-candidate parity sweep (GPU box): for every workload, random seeds and random unaligned
64-bit index windows, the verdicts of the JIT kernel (mgj_gen) and of the interpreter
(mg_eval_generated) against the C port's (oracle/bveval.c, test infrastructure).  Writes one JSON
line per workload and a total; any mismatch is reported with its first index.
usage: python tools/parity_sweep.py [windows-per-seed] [seeds]"""
import json
import random
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from mythril_amd import native, search, workloads  # noqa: E402
from oracle import cport  # noqa: E402

WIN = int(sys.argv[1]) if len(sys.argv) > 1 else 3
SEEDS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
N = 3000  # candidates per window (unaligned start, partial groups at both ends)

eng = native.Engine.get()
rng = random.Random(20261017)
total = {"candidates": 0, "mismatches": 0}
for name in workloads.WORKLOADS:
    t0 = time.time()
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    jh = eng.jit_compile(prog, gh, gen_verdicts=True)
    row = {"workload": name, "candidates": 0, "hits": 0, "jit_mismatch": 0, "interp_mismatch": 0, "first_bad": None}
    try:
        for _ in range(SEEDS):
            seed = rng.getrandbits(32)
            for _ in range(WIN):
                start = rng.getrandbits(63) | rng.getrandbits(6)
                _, _, want = cport.search(P.to_bytes(), blob, seed, start, N, threads=16, verdicts=True)
                vj = eng.jit_verdicts(jh, seed, start, N)
                vi, _ = eng.eval_generated(prog, gh, seed, start, N)
                bj = np.nonzero(vj != want)[0]
                bi = np.nonzero(vi != want)[0]
                row["candidates"] += N
                row["hits"] += int(want.sum())
                row["jit_mismatch"] += int(bj.size)
                row["interp_mismatch"] += int(bi.size)
                if (bj.size or bi.size) and row["first_bad"] is None:
                    row["first_bad"] = {"seed": seed, "index": start + int((bj if bj.size else bi)[0])}
    finally:
        eng.jit_free(jh)
        eng.free_gen(gh)
        eng.free(prog)
    row["seconds"] = round(time.time() - t0, 1)
    total["candidates"] += row["candidates"]
    total["mismatches"] += row["jit_mismatch"] + row["interp_mismatch"]
    print(json.dumps(row), flush=True)
print(json.dumps({"total": True, **total}), flush=True)
