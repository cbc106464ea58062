"""Row-major batched eval (bench.eval_roofline, default tier) at power-of-two candidate counts and
at counts just off them: does the SoA row pitch (= n) decide the HBM rate?  One JSON line each.

  python tools/eval_pitch.py [workload ...] > out.jsonl"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import bench
    from mythril_amd import native

    eng = native.Engine.get()
    names = sys.argv[1:] or ["token_transfer_underflow", "walletlibrary_kill"]
    for w in names:
        for n in (1 << 22, (1 << 22) + 64 * 13, (1 << 22) + 1024 * 7, (1 << 23), (1 << 23) + 64 * 13):
            r = bench.eval_roofline(eng, torch, w, n, "/nonexistent", tier="default")
            print(json.dumps({"workload": w, "n": n, "pitch_bytes": 4 * n, "tier": r["tier_built"],
                              "kernel_ms": r["kernel_ms"], "hbm_frac": r["hbm"]["frac"],
                              "gbs": r["hbm"]["achieved"]}), flush=True)


if __name__ == "__main__":
    main()
