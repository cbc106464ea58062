"""Run by tests/test_jit_isolation.py in its own process (the forced compiler abort turns the
JIT off for the process that sees it).  argv[1]: "host" (mg_program_jit_source, no GPU) or
"gpu" (a search whose compile aborts, then the same search answered on the interpreter).
Prints one JSON line."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from mythril_amd import native, search, workloads  # noqa: E402

mode = sys.argv[1]
out = {}
P, blob = search.prepare([c.raw for c in workloads.WORKLOADS["bectoken_batch_overflow"]()])
if mode == "host":
    native.jit_source(P.to_bytes(), blob, compile=True)
    out["pid_before"] = native.jit_helper_pid()
    os.environ["MYTHGPU_JITD_FAULT"] = "abort"
    try:
        native.jit_source(P.to_bytes(), blob, compile=True)
        out["fault_error"] = None
    except native.EngineError as e:
        out["fault_error"] = str(e)
    del os.environ["MYTHGPU_JITD_FAULT"]
    try:
        native.jit_source(P.to_bytes(), blob, compile=True)
        out["after_error"] = None
    except native.EngineError as e:
        out["after_error"] = str(e)
    out["pid_after"] = native.jit_helper_pid()
else:
    from mythril_amd.smt import Extract, symbol_factory

    eng = native.Engine.get()
    x = symbol_factory.BitVecSym("x", 256)
    k = symbol_factory.BitVecVal(0x9E3779B97F4A7C15F39CC0605CEDC835, 256)
    roots = [(Extract(19, 0, x * k) == symbol_factory.BitVecVal(0x12345, 20)).raw]  # ~2^-20: needs a search
    ref = search.search(eng, roots, timeout_s=30, jit="never", max_candidates=1 << 32)
    os.environ["MYTHGPU_JITD_FAULT"] = "abort"
    r1 = search.search(eng, roots, timeout_s=30, jit="always", max_candidates=1 << 32)  # compile aborts
    r2 = search.search(eng, roots, timeout_s=30, jit="auto", max_candidates=1 << 32)   # JIT off: interpreter
    out.update(ref=ref.index, always=r1.index, auto=r2.index, engines=[r1.engine, r2.engine],
               pid_after=native.jit_helper_pid(), model_ok=bool(r2.model and r2.model[0] == 1))
print(json.dumps(out), flush=True)
