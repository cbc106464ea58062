"""Per-phase wall time of the VMTests model read-back replay (GPU box): program load, JIT compile
(default tier = the first tier's eval kernel with watch rows, or O3), eval, free — where the replay's
seconds go.  python tools/vmtests_timing.py [n_vectors] > gpurun_out/vmtests_timing.json"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    from helpers import lift_literals, vmtest_cases
    from mythril_amd import native, ssa
    from mythril_amd.smt import terms as T

    n_max = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    eng = native.Engine.get()
    out = {}
    for o3 in (False, True):
        ph = {"prep": 0.0, "load": 0.0, "compile": 0.0, "eval": 0.0, "free": 0.0}
        n = 0
        for ci, (name, v, r) in enumerate(vmtest_cases()):
            keys = [int(k, 16) for k in v["post_storage"]]
            if not keys:
                continue
            if n >= n_max:
                break
            n += 1
            t0 = time.perf_counter()
            words = [r.storage_word(k).raw for k in keys]
            lifted, lits = lift_literals(words)
            P = ssa.flatten([T.BoolVal(True)], extra=lifted)
            P.set_watch([P.term_node[w.id] for w in lifted])
            soa = ssa.soa_from_assignments(P, [[0] * len(P.coords)])
            t1 = time.perf_counter()
            prog = eng.load(P.to_bytes())
            info = eng.info(prog)
            t2 = time.perf_counter()
            jh = eng.jit_compile(prog, 0, o3=o3)
            t3 = time.perf_counter()
            eng.jit_eval(jh, soa, 1, watch_words=info.watch_words)
            t4 = time.perf_counter()
            eng.jit_free(jh)
            eng.free(prog)
            t5 = time.perf_counter()
            for k, a, b in (("prep", t0, t1), ("load", t1, t2), ("compile", t2, t3), ("eval", t3, t4), ("free", t4, t5)):
                ph[k] += b - a
        out["o3" if o3 else "default"] = dict({k: round(v * 1e3 / max(n, 1), 2) for k, v in ph.items()}, vectors=n)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
