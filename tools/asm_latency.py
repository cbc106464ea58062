"""Latency of the JIT's first tier from submit to a loadable kernel, on fresh query shapes (new
sources each time, so no cache of any kind helps): the bench's hard needle with a different needle
constant per sample; alone, and with an O3 compile of the same query in flight on the other lane.
Stage split (emission / helper assemble+link / module load) with MYTHGPU_JIT_TIMING=1 on stderr.

  MYTHGPU_JIT_TIMING=1 python tools/asm_latency.py > gpurun_out/asm_latency.jsonl
"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
os.environ.setdefault("AMD_COMGR_CACHE", "0")
os.environ.setdefault("MYTHGPU_JIT_DISK_CACHE", "0")


def main():
    from mythril_amd import native, search, workloads
    from mythril_amd.smt import Extract, symbol_factory

    eng = native.Engine.get()
    cs = workloads.WORKLOADS["token_transfer_underflow"]()
    x = symbol_factory.BitVecSym("lat_x", 256)
    k = symbol_factory.BitVecVal(0x9E3779B97F4A7C15F39CC0605CEDC835, 256)

    def shape(i):
        needle = Extract(23, 0, x * k) == symbol_factory.BitVecVal(0xA5C3E1 ^ i, 24)
        P, blob = search.prepare([c.raw for c in cs] + [needle.raw])
        prog = eng.load(P.to_bytes())
        return prog, eng.load_gen(prog, blob)

    # start both helpers first (their spawn is a once-per-process cost)
    prog, gh = shape(10_000)
    eng.jit_free(eng.jit_compile(prog, gh, asm=True))
    eng.jit_free(eng.jit_compile(prog, gh))
    for mode in ("alone", "beside_o3"):
        ts = []
        for i in range(8):
            prog, gh = shape(i + (100 if mode == "beside_o3" else 0))
            o3 = eng.jit_compile_async(prog, gh) if mode == "beside_o3" else None
            t = time.perf_counter()
            tk = eng.jit_compile_async(prog, gh, asm=True)
            h = None
            while h is None:
                h = eng.jit_poll(tk, 1)
            ts.append((time.perf_counter() - t) * 1e3)
            eng.jit_free(h)
            if o3 is not None:
                eng.jit_cancel(o3)
            eng.free_gen(gh)
            eng.free(prog)
        print(json.dumps({"first_tier_submit_to_ready_ms": mode, "median": statistics.median(ts),
                          "min": min(ts), "max": max(ts), "samples": [round(v, 2) for v in ts]}), flush=True)


if __name__ == "__main__":
    main()
