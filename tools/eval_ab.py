"""Batched eval HBM fractions (bench.eval_roofline) of C2 and C4, row-major and tiled, default tier
and the first tier, one JSON line each; environment variants go in the environment, --tag labels them.

  python tools/eval_ab.py --tag T [--n N] > out.jsonl"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="base")
    ap.add_argument("--n", type=int, default=1 << 22)
    a = ap.parse_args()
    import torch
    import bench
    from mythril_amd import native

    eng = native.Engine.get()
    for w in ("token_transfer_underflow", "walletlibrary_kill"):
        for tiled in (False, True):
            for tier in ("asm",):
                r = bench.eval_roofline(eng, torch, w, a.n, "/nonexistent", tiled=tiled, tier=tier)
                print(json.dumps({"tag": a.tag, "workload": w, "tiled": tiled, "tier": r["tier_built"],
                                  "kernel_ms": r["kernel_ms"], "hbm_frac": r["hbm"]["frac"],
                                  "sat_fraction": r["sat_fraction"], "sha": r["jit_source_sha16"]}), flush=True)


if __name__ == "__main__":
    main()
