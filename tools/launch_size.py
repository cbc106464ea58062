"""Search-kernel rate against launch size (C2 is quoted at 2^24 candidates per launch).
For each launch size, 16 seeds x one launch each of the workload's O3 kernel (no early exit):
mean kernel time (HIP events) and wall time per launch, candidates/s.  The engine's blocks-per-CU
rule is what is measured; run once per MYTHGPU_JIT_MIN_GROUPS / MYTHGPU_JIT_BPC setting to compare.

  python tools/launch_size.py [workload] [--asm] > gpurun_out/launch_size.jsonl
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from mythril_amd import native, search, workloads

    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    name = args[0] if args else "token_transfer_underflow"
    eng = native.Engine.get()
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    jit = eng.jit_compile(prog, gh, asm="--asm" in sys.argv)
    eng.jit_search(jit, 1, 0, 1 << 24, early_exit=False)
    for lg in (20, 22, 24, 26, 28):
        n = 1 << lg
        eng.reset_stats()
        t = time.perf_counter()
        for seed in range(1, 17):
            eng.jit_search(jit, seed, 0, n, early_exit=False)
        wall = (time.perf_counter() - t) / 16
        st = eng.stats()
        km = st.kernel_ms_total / max(st.launches, 1)
        print(json.dumps({"workload": name, "tier": "asm" if "--asm" in sys.argv else "o3", "log2_launch": lg,
                          "kernel_ms": round(km, 4), "wall_ms": round(wall * 1e3, 4),
                          "g_per_s_kernel": round(n / km / 1e6, 2), "g_per_s_wall": round(n / wall / 1e9, 2),
                          "min_groups": os.environ.get("MYTHGPU_JIT_MIN_GROUPS", "16"),
                          "bpc": os.environ.get("MYTHGPU_JIT_BPC", "auto")}), flush=True)


if __name__ == "__main__":
    main()
