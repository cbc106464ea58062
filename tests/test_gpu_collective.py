"""The split search's exchange as one RCCL all-reduce(min) (engine.hip rccl_ready /
rccl_first_hit_min, ``MYTHGPU_COLLECTIVE``).

On the one-GPU box the all-reduce runs over a one-rank communicator (``MYTHGPU_COLLECTIVE=rccl-force``):
librccl is loaded, the communicator built, the all-reduce queued on the engine's stream between
the search kernel and the read-back — and the first hits and counts equal the host reduction's
and the C port's on the same windows.  A mask of logical devices on one GPU cannot form an RCCL
communicator and keeps the host reduction (``mg_collective_kind`` 0).  The multi-GPU case needs
distinct physical GPUs (the driver's 8-GPU node), which no test here can reach."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

SCRIPT = r"""
import json
from mythril_amd import native, search, workloads
eng = native.Engine.get()
out = {"kind": eng.lib.mg_collective_kind()}
rows = []
for w in ("token_transfer_underflow", "bectoken_batch_overflow", "walletlibrary_kill"):
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[w]()])
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    jh = eng.jit_compile(prog, gh, asm=True)
    for start, n, early in ((0, 1 << 16, True), (12345, 1 << 20, False), ((1 << 40) + 7, 1 << 18, False)):
        rows.append([w, start, n, early, list(eng.jit_search(jh, 7, start, n, early_exit=early))])
    eng.jit_free(jh)
out["rows"] = rows
print(json.dumps(out))
"""


def _run(**env):
    e = dict(os.environ, PYTHONPATH=str(ROOT))
    e.update(env)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_rccl_first_hit_equals_host_reduction():
    from mythril_amd import search, workloads
    from oracle import cport

    host = _run()
    rccl = _run(MYTHGPU_COLLECTIVE="rccl-force")
    assert host["kind"] == 0
    assert rccl["kind"] == 1, "librccl did not load or the one-rank communicator failed"
    # first hits everywhere; counts only for full sweeps (an early-exit search's count depends on when
    # the waves above the first hit saw it)
    for a, b in zip(rccl["rows"], host["rows"]):
        assert a[:4] == b[:4] and a[4][0] == b[4][0] and (a[3] or a[4][1] == b[4][1]), (a, b)
    for w, start, n, early, (first, hits) in rccl["rows"]:
        if early:
            continue
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[w]()])
        want = cport.search(P.to_bytes(), blob, 7, start, n, threads=16)[:2]
        assert (first, hits) == want, (w, start, n)


@pytest.mark.gpu
def test_logical_devices_keep_the_host_reduction():
    """k logical devices on one GPU: no communicator (duplicate device), host reduction, same answers."""
    virt = _run(MYTHGPU_COLLECTIVE="rccl", MYTHGPU_VIRTUAL_DEVICES="2", MYTHGPU_SPLIT_MIN="4096")
    host = _run()
    assert virt["kind"] == 0
    for a, b in zip(virt["rows"], host["rows"]):
        assert a[4][0] == b[4][0] and (a[3] or a[4][1] == b[4][1]), (a, b)
