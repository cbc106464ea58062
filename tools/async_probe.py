import sys, time, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tools")
import os
from mythril_amd import native, search, ssa
import stream_bench
eng = native.Engine.get()
qs = dict(stream_bench.stream_queries("token_transfer_underflow"))
roots = [c.raw for c in qs["hard"]]
from mythril_amd.partition import partition
bs = partition(roots)
print("buckets", len(bs), [len(b) for b in bs])
big = max(bs, key=len)
P, blob = search.prepare(big)
prog = eng.load(P.to_bytes()); gh = eng.load_gen(prog, blob)
t = time.perf_counter(); h = eng.jit_compile(prog, gh); print("sync compile ms", (time.perf_counter()-t)*1e3); eng.jit_free(h)
os.environ["AMD_COMGR_CACHE"] = "0"
# async while idle
t = time.perf_counter(); tk = eng.jit_compile_async(prog, gh); h = eng.jit_poll(tk, wait_ms=-1); print("async idle ms (cache hit)", (time.perf_counter()-t)*1e3); eng.jit_free(h)
# async while interp runs 10ms chunks
for n in (1<<22, 1<<20):
    # new source to avoid code cache: different program (drop a root)
    P2, blob2 = search.prepare(big[:-1] if n == (1<<22) else big[1:])
    prog2 = eng.load(P2.to_bytes()); gh2 = eng.load_gen(prog2, blob2)
    t = time.perf_counter(); tk = eng.jit_compile_async(prog2, gh2); launches = 0; h = None
    while h is None and time.perf_counter() - t < 2.0:
        eng.search(prog2, gh2, 1, launches * n, n, early_exit=True); launches += 1
        h = eng.jit_poll(tk)
    print(f"async under load (chunk {n}) ready after ms", (time.perf_counter()-t)*1e3, "launches", launches, "got", h is not None)
    if h: eng.jit_free(h)
