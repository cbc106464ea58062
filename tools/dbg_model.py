import sys, os, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.getcwd() + "/tests")
from mythril_amd import native, search, workloads
from oracle.bv import evaluate
from helpers import OracleModel
eng = native.Engine.get()
for trial in range(3):
    for name in ["token_transfer_underflow", "suicide_kill"]:
        roots = [c.raw for c in workloads.WORKLOADS[name]()]
        res = search.search(eng, roots, max_candidates=1 << 28, timeout_s=60)
        ver, scalars, arrays, funcs, P = res.model
        m = OracleModel(scalars, arrays, funcs)
        oks = [evaluate(r, m) for r in roots]
        print(json.dumps({"trial": trial, "name": name, "index": res.index, "engine": res.engine, "ver": ver, "roots_ok": oks, "timing": getattr(res, "timing", None)}, default=str), flush=True)
