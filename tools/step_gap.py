"""Per-call wall time of jit_search vs the kernel's own HIP-event time (diagnostic)."""
import sys
import time

w = sys.argv[1] if len(sys.argv) > 1 else "token_transfer_underflow"
if "torchfirst" in sys.argv[2:]:
    import torch

    torch.cuda.set_device(0)
    x = torch.zeros(1, device="cuda")

from mythril_amd import native, search, ssa, workloads  # noqa: E402

C = 1 << 26
eng = native.Engine.get()
roots = [c.raw for c in workloads.WORKLOADS[w]()]
P = ssa.flatten(roots)
blob = search.default_generator(P, roots=roots).blob()
prog = eng.load(P.to_bytes())
gh = eng.load_gen(prog, blob)
jit = eng.jit_compile(prog, gh)
if "torchlate" in sys.argv[2:]:
    import torch

    torch.cuda.set_device(0)
    x = torch.zeros(1, device="cuda")
for s in range(int(sys.argv[3]) if len(sys.argv) > 3 else 8):
    t = time.perf_counter()
    idx, nh = eng.jit_search(jit, 0x6D797468, s * C, C, early_exit=False)
    wall = (time.perf_counter() - t) * 1e3
    print(f"step {s}: wall {wall:.3f} ms kernel {eng.stats().last_kernel_ms:.3f} ms hits {nh}", flush=True)
libs = sorted({l.split()[-1] for l in open("/proc/self/maps") if any(k in l for k in ("hiprtc", "comgr", "amdhip64", "hsa-runtime"))})
print("\n".join(libs))
