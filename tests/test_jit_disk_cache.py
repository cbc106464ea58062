"""The engine's on-disk JIT code-object cache (``jit.cpp: jit_compile``, MYTHGPU_JIT_DISK_CACHE).

A query kernel compiled by one process loads from the cache in the next, without the compiler
helper; a damaged cache file is a miss (recompiled and rewritten), never an error; a different
compile environment is a different key.  Host only: comgr compiles for gfx950 without a GPU."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

from mythril_amd import search, workloads

ROOT = Path(__file__).resolve().parent.parent

SCRIPT = r"""
from mythril_amd import native, search, workloads
cs = workloads.WORKLOADS["bectoken_batch_overflow"]()
P, blob = search.prepare([c.raw for c in cs])
native.jit_source(P.to_bytes(), blob, compile=True)
"""


def _compile(cache: Path, **env):
    e = dict(os.environ, PYTHONPATH=str(ROOT), MYTHGPU_JIT_DISK_CACHE=str(cache), MYTHGPU_JIT_TIMING="1")
    e.update(env)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stderr


@pytest.fixture(scope="module", autouse=True)
def _built():
    from mythril_amd import build

    build.build()


def test_second_process_loads_the_code_object_from_disk(tmp_path):
    cache = tmp_path / "jit"
    err = _compile(cache)
    assert "stored in the disk cache" in err and "from the disk cache" not in err
    files = list(cache.glob("*.co"))
    assert len(files) == 1
    assert files[0].read_bytes()[24:28] == b"\x7fELF"
    # the second process never starts the compiler: the helper binary named here does not exist
    err = _compile(cache, MYTHGPU_JITD=str(tmp_path / "no_such_helper"))
    assert "from the disk cache" in err and "compiling in-process" not in err
    assert not list(cache.glob("*.tmp.*"))


def test_damaged_entry_is_a_miss_and_is_rewritten(tmp_path):
    cache = tmp_path / "jit"
    _compile(cache)
    (f,) = cache.glob("*.co")
    good = f.read_bytes()
    f.write_bytes(good[:24] + b"garbage")
    err = _compile(cache)
    assert "stored in the disk cache" in err and "from the disk cache" not in err
    assert f.read_bytes() == good


def test_compile_environment_is_part_of_the_key(tmp_path):
    cache = tmp_path / "jit"
    _compile(cache)
    err = _compile(cache, MYTHGPU_JIT_FAST="0")  # a different compile: its own entry
    assert "stored in the disk cache" in err
    assert len(list(cache.glob("*.co"))) == 2
    err = _compile(cache, AMD_COMGR_CACHE="0")  # comgr's cache switch decides nothing in the code
    assert "from the disk cache" in err


def test_cache_off(tmp_path):
    err = _compile(Path("0"))
    assert "disk cache" not in err


GPU_SCRIPT = r"""
import json
from mythril_amd import native, search, workloads
eng = native.Engine.get()
cs = workloads.WORKLOADS["bectoken_batch_overflow"]()
P, blob = search.prepare([c.raw for c in cs])
prog = eng.load(P.to_bytes())
gh = eng.load_gen(prog, blob)
jit = eng.jit_compile(prog, gh)
print(json.dumps(list(eng.jit_search(jit, 5, (1 << 40) + 12345, 1 << 18, early_exit=False))))
"""


@pytest.mark.gpu
def test_cached_code_object_searches_like_a_fresh_compile(tmp_path):
    """C3 (BECToken batchOverflow): the kernel a second process loads from the disk cache finds
    the same first hit and hit count as the freshly compiled one, and both equal the C port's."""
    from oracle import cport

    cache = tmp_path / "jit"
    env = dict(os.environ, PYTHONPATH=str(ROOT), MYTHGPU_JIT_DISK_CACHE=str(cache), MYTHGPU_JIT_TIMING="1")
    outs = []
    for _ in range(2):
        r = subprocess.run([sys.executable, "-c", GPU_SCRIPT], env=env, capture_output=True, text=True, timeout=200)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append((r.stdout.strip().splitlines()[-1], r.stderr))
    assert "stored in the disk cache" in outs[0][1]
    assert "from the disk cache" in outs[1][1]
    assert outs[0][0] == outs[1][0]
    P, blob = search.prepare([c.raw for c in workloads.WORKLOADS["bectoken_batch_overflow"]()])
    want = cport.search(P.to_bytes(), blob, 5, (1 << 40) + 12345, 1 << 18, threads=16)[:2]
    assert json.loads(outs[1][0]) == list(want)
