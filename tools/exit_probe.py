"""Exit probe (GPU box): submit an asynchronous compile of the C4 search kernel and return from
``main`` at once, so the process exits with the compile in flight.  This is the situation in
which a stream run once ended in an LLVM fatal error at exit (commits 0546a51, 56335f1).

usage: python tools/exit_probe.py [--no-atexit]
  --no-atexit   unregister the Python atexit handler that stops the engine (native.py), leaving
                only the C-level exit path — the configuration of the original abort
Prints one JSON line (what was submitted) before returning; the caller records the rc and stderr.
"""
import atexit
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from mythril_amd import native, search, workloads  # noqa: E402


def main():
    eng = native.Engine.get()
    if "--no-atexit" in sys.argv:
        atexit.unregister(native._shutdown_at_exit)
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS["walletlibrary_kill"]()])
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    t = time.perf_counter()
    ticket = eng.jit_compile_async(prog, gh)
    # a few ms in: the compile thread is inside the compiler when main returns
    time.sleep(0.02)
    print(json.dumps({"probe": "exit with compile in flight", "ticket": ticket,
                      "atexit_handler": "--no-atexit" not in sys.argv,
                      "jit_helper": getattr(native, "jit_helper_pid", lambda: None)(),
                      "submitted_ms_ago": round((time.perf_counter() - t) * 1e3, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
