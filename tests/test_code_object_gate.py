"""The JIT load gate (``jit.cpp: jit_check_code_object``, ``mg_code_object_check``).

Every code object the engine would hand to ``hipModuleLoadData`` — compiled by comgr or read from
the disk cache — passes a check of its AMDHSA kernel descriptors first: a kernel with a dynamic
stack, or with more private (scratch) segment per lane than ``MYTHGPU_JIT_PRIVATE_CAP`` (default
16 KiB), or more LDS than a CU has, is refused with ``MG_E_UNSUPPORTED``.  The search then stays on
the interpreter and the ``get_model`` hook on z3 (``mythril/support/model.py:15-49``), instead of a
GPU fault: round 5's read-back kernel compiled at -O0 kept 52 KB per lane on a dynamic stack and
faulted (``profiles/r05n_gpu_pytest_O0_fault.log``).

Host only: comgr compiles for gfx950 without a GPU.
"""
import ctypes as C
import os
import struct
import subprocess
import sys
from pathlib import Path

import pytest

from mythril_amd import native

ROOT = Path(__file__).resolve().parent.parent

SCRIPT = r"""
import sys
from mythril_amd import native, search, workloads
cs = workloads.WORKLOADS[sys.argv[1]]()
P, blob = search.prepare([c.raw for c in cs])
try:
    native.jit_source(P.to_bytes(), blob if sys.argv[2] == "search" else None, compile=True)
    print("COMPILED")
except native.EngineError as e:
    print("REFUSED", e)
"""


def _compile(cache: Path, workload: str, kind: str, **env):
    e = dict(os.environ, PYTHONPATH=str(ROOT), MYTHGPU_JIT_DISK_CACHE=str(cache))
    e.update(env)
    r = subprocess.run([sys.executable, "-c", SCRIPT, workload, kind], env=e, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.strip().splitlines()[-1]


def check(code: bytes):
    lib = native.load_library()
    k, p, g, d = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
    rc = lib.mg_code_object_check(code, len(code), C.byref(k), C.byref(p), C.byref(g), C.byref(d))
    return rc, k.value, p.value, g.value, d.value


def kd_offsets(code: bytes):
    """File offsets of every ``*.kd`` kernel descriptor (ELF64 little-endian, .symtab), restated
    independently of the engine's parser."""
    shoff, = struct.unpack_from("<Q", code, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", code, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", code, shoff + i * shentsize) for i in range(shnum)]
    out = []
    for name, typ, flags, addr, off, size, link, info, align, entsize in secs:
        if typ != 2:  # SHT_SYMTAB
            continue
        stroff = secs[link][4]
        for i in range(size // entsize):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", code, off + i * entsize)
            end = code.index(b"\0", stroff + st_name)
            if code[stroff + st_name:end].endswith(b".kd"):
                sec = secs[st_shndx]
                out.append(sec[4] + (st_value - sec[3]))
    return out


@pytest.fixture(scope="module", autouse=True)
def _built():
    from mythril_amd import build

    build.build()


def test_o3_kernels_pass_and_o0_dynamic_stack_is_refused(tmp_path):
    """The O3 search kernel loads; the same kernel at -O0 (MYTHGPU_JIT_OPT=0: LLVM's -O0 code puts
    its frames on a dynamic stack) is refused before any load, and nothing is cached for it."""
    c3, c0 = tmp_path / "o3", tmp_path / "o0"
    assert _compile(c3, "bectoken_batch_overflow", "search") == "COMPILED"
    (co,) = c3.glob("*.co")
    rc, kernels, priv, lds, dyn = check(co.read_bytes()[24:])
    assert (rc, kernels, priv, dyn) == (0, 1, 0, 0) and lds < 160 * 1024
    out = _compile(c0, "bectoken_batch_overflow", "search", MYTHGPU_JIT_OPT="0")
    assert out.startswith("REFUSED") and "dynamic stack" in out, out
    assert not list(c0.glob("*.co")), "a refused code object must not reach the disk cache"


def test_private_segment_cap(tmp_path):
    """An -O0 eval kernel has a static private segment (KBs per lane, no dynamic stack): it loads
    under the default cap and is refused under a smaller MYTHGPU_JIT_PRIVATE_CAP."""
    out = _compile(tmp_path / "a", "suicide_kill", "eval", MYTHGPU_JIT_OPT="0")
    assert out == "COMPILED", out
    (co,) = (tmp_path / "a").glob("*.co")
    rc, _, priv, _, dyn = check(co.read_bytes()[24:])
    assert rc == 0 and dyn == 0 and 1024 < priv <= 16384, priv
    out = _compile(tmp_path / "b", "suicide_kill", "eval", MYTHGPU_JIT_OPT="0", MYTHGPU_JIT_PRIVATE_CAP="1024")
    assert out.startswith("REFUSED") and "private segment" in out, out


def test_descriptor_fields_and_a_poisoned_disk_cache_entry(tmp_path):
    """The parser reads the descriptor fields the runtime sizes scratch from: setting bit 11
    (USES_DYNAMIC_STACK) of kernel_code_properties, or a 64 KiB private segment, in a good object
    makes it refused; such an object found in the disk cache (written by a build without the gate)
    is refused and evicted, and the next compile stores a good one again."""
    cache = tmp_path / "c"
    assert _compile(cache, "etherstore_reentrancy", "search") == "COMPILED"
    (co,) = cache.glob("*.co")
    raw = co.read_bytes()
    code = raw[24:]
    (kd,) = kd_offsets(code)
    props, = struct.unpack_from("<H", code, kd + 56)
    dyn = bytearray(code)
    struct.pack_into("<H", dyn, kd + 56, props | (1 << 11))
    assert check(bytes(dyn))[0] == native.MG_E_UNSUPPORTED and check(bytes(dyn))[4] == 1
    big = bytearray(code)
    struct.pack_into("<I", big, kd + 4, 65536)
    rc, _, priv, _, _ = check(bytes(big))
    assert rc == native.MG_E_UNSUPPORTED and priv == 65536
    assert check(b"\x7fELF" + b"\0" * 100)[0] == native.MG_E_INVALID
    co.write_bytes(raw[:24] + bytes(dyn))
    out = _compile(cache, "etherstore_reentrancy", "search")
    assert out.startswith("REFUSED") and "dynamic stack" in out, out
    assert not co.exists(), "the poisoned entry is evicted"
    assert _compile(cache, "etherstore_reentrancy", "search") == "COMPILED"
    assert check(co.read_bytes()[24:])[0] == 0


@pytest.mark.gpu
def test_refused_o3_kernel_on_the_gpu(monkeypatch):
    """On the box: an O3 compile that produces a dynamic-stack kernel (-O0) fails its request with
    MG_E_UNSUPPORTED before any module load, ``mg_stats`` counts it, and the engine keeps working —
    the same query is answered by the interpreter and the first tier, whose model the oracle
    accepts."""
    from mythril_amd import search, workloads
    from oracle.bv import OracleModel, evaluate

    eng = native.Engine.get()
    roots = [c.raw for c in workloads.WORKLOADS["etherstore_reentrancy"]()]
    P, blob = search.prepare(roots)
    monkeypatch.setenv("MYTHGPU_JIT_OPT", "0")
    monkeypatch.setenv("MYTHGPU_JIT_DISK_CACHE", "0")
    eng.cache_clear()
    before = eng.stats().jit_refused
    prog = eng.load(P.to_bytes())
    gen = eng.load_gen(prog, blob)
    try:
        with pytest.raises(native.EngineUnsupported, match="dynamic stack"):
            eng.jit_compile(prog, gen)
    finally:
        eng.free_gen(gen)
        eng.free(prog)
    assert eng.stats().jit_refused == before + 1
    res = search.search(eng, roots, max_candidates=1 << 24, timeout_s=30)
    assert res.index is not None
    ver, scalars, arrays, funcs, _ = res.model
    m = OracleModel(scalars, arrays, funcs)
    assert ver == 1 and all(evaluate(r, m) == 1 for r in roots)
    monkeypatch.delenv("MYTHGPU_JIT_OPT")
    eng.cache_clear()
