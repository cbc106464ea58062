"""The first tier's round-6 code paths against their predecessors on the GPU: limb-pair dictionary
reads (``ds_read_b64``) vs one limb per read (``MYTHGPU_JIT_ASM_LDS_B32=1``), dictionary-index
compares vs the XOR/OR reduction (``MYTHGPU_JIT_ASM_NO_DICT_EQ=1``), the specialiser's
NOT(compare) folding vs the two instructions (``MYTHGPU_FOLD_NOT=0``), and the generator's folded
key, one-multiply dictionary index and one-instruction ALIGNED offset vs their first forms.  Each variant runs in its own
process (the switches are read once) over the same full-sweep windows; every first hit and hit
count equals the C port's (``oracle/bveval.c``), so each variant is checked, not only compared.

Reference anchor: a candidate's verdict is ``Model.eval(And(constraints), model_completion=True)``
(``mythril/laser/smt/model.py:45-59``) over the GEN3 candidate stream."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
WORKLOADS = ("suicide_kill", "token_transfer_underflow", "walletlibrary_kill")
WINDOWS = ((0, 1 << 18), (987654321, 1 << 20), ((1 << 41) + 3, 1 << 18))

SCRIPT = r"""
import json, sys
from mythril_amd import native, search, workloads
eng = native.Engine.get()
rows = []
for w in sys.argv[1].split(","):
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[w]()])
    prog = eng.load(P.to_bytes())
    gh = eng.load_gen(prog, blob)
    jh = eng.jit_compile(prog, gh, asm=True)
    assert eng.jit_layout(jh)[0] & native.MG_JIT_ASM, "not the first tier"
    for start, n in json.loads(sys.argv[2]):
        rows.append([w, start, n, list(eng.jit_search(jh, 7, start, n, early_exit=False))])
    eng.jit_free(jh)
print(json.dumps(rows))
"""


def _run(env):
    e = dict(os.environ, PYTHONPATH=str(ROOT))
    e.update(env)
    r = subprocess.run([sys.executable, "-c", SCRIPT, ",".join(WORKLOADS), json.dumps(WINDOWS)], env=e,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [
    {},
    {"MYTHGPU_JIT_ASM_LDS_B32": "1"},
    {"MYTHGPU_JIT_ASM_NO_DICT_EQ": "1"},
    {"MYTHGPU_FOLD_NOT": "0"},
    {"MYTHGPU_JIT_ASM_NO_KFOLD": "1", "MYTHGPU_JIT_ASM_NO_MULHI24": "1", "MYTHGPU_JIT_ASM_ALIGNED_MAD": "0"},
], ids=["default", "lds_b32", "no_dict_eq", "no_fold_not", "generator_v1"])
def test_first_tier_variant_matches_c_port(variant):
    from mythril_amd import search, workloads
    from oracle import cport

    rows = _run(dict(variant, MYTHGPU_JIT_DISK_CACHE="0"))
    assert len(rows) == len(WORKLOADS) * len(WINDOWS)
    for w, start, n, (first, hits) in rows:
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[w]()])
        want = cport.search(P.to_bytes(), blob, 7, start, n, threads=16)[:2]
        assert (first, hits) == want, (variant, w, start, n, (first, hits), want)
