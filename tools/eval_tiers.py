"""Batched verdict eval (``Model.eval`` batched, ``laser/smt/model.py:45-59``) on every workload,
both compiled tiers (O3, first tier) and both SoA layouts, plus the tier the engine picks by
default (``mg_jit_compile_ex`` with no tier flag): one JSON line per kernel, as bench.py's
``roofline_eval`` entries.  Usage: ``python tools/eval_tiers.py [n] > out.jsonl``."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import bench
    from mythril_amd import native, workloads

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    eng = native.Engine.get()
    for w in workloads.WORKLOADS:
        for tier in ("default", "o3", "asm"):
            for tiled in (False, True):
                try:
                    r = bench.eval_roofline(eng, torch, w, n, str(ROOT / "profiles"), tier=tier, tiled=tiled)
                except native.EngineUnsupported as e:
                    r = {"workload": w, "tier": tier, "tiled": tiled, "unsupported": str(e)}
                r["requested_tier"] = tier
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
