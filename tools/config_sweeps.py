"""Every BASELINE config at the candidate count SURVEY.md §8(d) names for it, on the GPUs this
process opens (GPU box):  python tools/config_sweeps.py [--gpus N] > gpurun_out/config_sweeps.jsonl

  C2 token.sol / etherstore.sol   2^24 candidates per launch, seeds 1..16
  C3 BECToken batchOverflow       2^30 candidates
  C4 WalletLibrary -t 3           2^32 candidates
  C5 SHA3-keyed mapping           10^10 candidates
  C1 suicide.sol -t 2             the query shape the reference run dumps, 2^30 candidates

Each sweep runs the query's compiled search kernel (the product's mg_jit_search) over the whole
range with no early exit, in launches of at most 2^28 candidates (C5: 2^24), and reports the wall
time, the rate, the satisfying-candidate count and the lowest satisfying index; then the product
path search.search answers the query from index 0 (time to first model).  Multi-seed configs
are also swept as one mg_jit_search_many call (candidates_per_s_many: best of three).  --gpus N opens N devices
in this process (mg_init mask): every launch is split over them inside the shim."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

CONFIGS = [
    ("C1", "suicide_kill", 1 << 30, [0x6D797468]),
    ("C2", "token_transfer_underflow", 1 << 24, list(range(1, 17))),
    ("C2", "etherstore_reentrancy", 1 << 24, list(range(1, 17))),
    ("C3", "bectoken_batch_overflow", 1 << 30, [0x6D797468]),
    ("C4", "walletlibrary_kill", 1 << 32, [0x6D797468]),
    ("C5", "sha3_keyed_mapping", 10 ** 10, [0x6D797468]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--only", default="", help="comma-separated workload names")
    args = ap.parse_args()
    if args.gpus > 1:
        os.environ["MYTHGPU_DEVICES"] = ",".join(str(d) for d in range(args.gpus))
    from mythril_amd import native, search, workloads

    eng = native.Engine.get()
    if eng.n_devices != args.gpus:
        print(f"config_sweeps: engine opened {eng.n_devices} device(s), wanted {args.gpus}", file=sys.stderr)
        sys.exit(2)
    only = set(filter(None, args.only.split(",")))
    for cfg, name, n, seeds in CONFIGS:
        if only and name not in only:
            continue
        roots = [c.raw for c in workloads.WORKLOADS[name]()]
        P, blob = search.prepare(roots)
        prog = eng.load(P.to_bytes())
        gh = eng.load_gen(prog, blob)
        t = time.perf_counter()
        jit = eng.jit_compile(prog, gh)
        compile_ms = (time.perf_counter() - t) * 1e3
        chunk = (1 << 24) if name == "sha3_keyed_mapping" else (1 << 28)
        eng.jit_search(jit, seeds[0], 0, min(n, chunk), early_exit=False)  # warm-up (module, caches)
        per_seed = []
        for seed in seeds:
            t = time.perf_counter()
            first, hits, start = None, 0, 0
            while start < n:
                c = min(chunk, n - start)
                idx, nh = eng.jit_search(jit, seed, start, c, early_exit=False)
                if idx is not None and first is None:
                    first = idx
                hits += nh
                start += c
            per_seed.append({"seed": seed, "s": time.perf_counter() - t, "hits": hits, "first": first})
        # the same sweep as one mg_jit_search_many call: every (seed, chunk) launch queued back to back
        # over four streams, one wait (the host round trip per launch above is what a 2^24 launch pays)
        many_s = None
        if len(seeds) > 1:
            ss, st, ct = [], [], []
            for seed in seeds:
                for a in range(0, n, chunk):
                    ss.append(seed)
                    st.append(a)
                    ct.append(min(chunk, n - a))
            eng.jit_search_many(jit, ss[:4], st[:4], ct[:4])  # warm-up (streams, slots)
            reps = []
            for _ in range(3):
                t = time.perf_counter()
                res_many = eng.jit_search_many(jit, ss, st, ct)
                reps.append(time.perf_counter() - t)
            many_s = min(reps)
            assert sum(h for _, h in res_many) == sum(r["hits"] for r in per_seed)
        eng.jit_free(jit)
        eng.free_gen(gh)
        eng.free(prog)
        secs = sum(r["s"] for r in per_seed)
        t = time.perf_counter()
        res = search.search(eng, roots, seed=seeds[0], max_candidates=1 << 36, timeout_s=30)
        ttfm_ms = (time.perf_counter() - t) * 1e3
        print(json.dumps({
            "config": cfg, "workload": name, "n_gpus": args.gpus, "candidates_per_seed": n, "seeds": len(seeds),
            "wall_s": round(secs, 4), "candidates_per_s": n * len(seeds) / secs,
            "hits": sum(r["hits"] for r in per_seed), "first_hit_seed0": per_seed[0]["first"],
            "many_wall_s": None if many_s is None else round(many_s, 5),
            "candidates_per_s_many": None if many_s is None else n * len(seeds) / many_s,
            "jit_compile_ms": round(compile_ms, 1), "time_to_first_model_ms": round(ttfm_ms, 3),
            "ttfm_index": res.index, "ttfm_engine": res.engine,
        }), flush=True)


if __name__ == "__main__":
    main()
