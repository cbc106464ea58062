"""Search-kernel rates of both compiled tiers on every workload (full evaluation, no early exit),
from the engine's HIP events: one JSON line per (workload, tier).  Environment variants go in the
environment; ``--tag`` labels the lines.

  python tools/tier_rates.py [--tag T] [--n N] [--tiers asm,o3] [workload ...] > out.jsonl"""
import argparse
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="base")
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--tiers", default="asm,o3")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("workloads", nargs="*")
    a = ap.parse_args()
    from mythril_amd import native, search, workloads

    eng = native.Engine.get()
    names = a.workloads or list(workloads.WORKLOADS)
    for w in names:
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[w]()])
        prog = eng.load(P.to_bytes())
        gh = eng.load_gen(prog, blob)
        n = a.n if w != "sha3_keyed_mapping" else min(a.n, 1 << 24)
        for tier in a.tiers.split(","):
            try:
                jh = eng.jit_compile(prog, gh, asm=tier == "asm")
            except native.EngineUnsupported as e:
                print(json.dumps({"workload": w, "tier": tier, "tag": a.tag, "unsupported": str(e)}), flush=True)
                continue
            src = native.jit_asm(P.to_bytes(), blob) if tier == "asm" else native.jit_source(P.to_bytes(), blob)
            eng.jit_search(jh, 7, 0, n, early_exit=False)
            eng.reset_stats()
            res = None
            for r in range(a.reps):
                res = eng.jit_search(jh, 7, (r + 1) * n, n, early_exit=False)
            st = eng.stats()
            ms = st.kernel_ms_total / max(st.launches, 1)
            print(json.dumps({"workload": w, "tier": tier, "tag": a.tag, "n": n, "kernel_ms": ms,
                              "candidates_per_s": n / (ms * 1e-3), "last": list(res),
                              "jit_source_sha16": hashlib.sha256(src.encode()).hexdigest()[:16]}), flush=True)
            eng.jit_free(jh)
        eng.free_gen(gh)
        eng.free(prog)


if __name__ == "__main__":
    main()
