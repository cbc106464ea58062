"""Build the in-tree native library ``mythril_amd/libmythgpu.so`` for gfx950.

``hipcc --offload-arch=gfx950`` cross-compiles here (no GPU needed); the built
``.so`` is git-ignored but travels to the GPU box with the tree snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
LIB = PKG / "libmythgpu.so"
JITD = PKG / "mythgpu_jitd"  # the JIT compiler process (csrc/jitd.cpp), next to the library
JITD_SOURCES = [CSRC / "jitd.cpp", CSRC / "jit.cpp", CSRC / "program.cpp"]

SOURCES = [CSRC / "engine.hip", CSRC / "program.cpp", CSRC / "jit.cpp", CSRC / "jit_asm.cpp"]
HEADERS = [CSRC / "bv_device.h", CSRC / "keccak_device.h", CSRC / "gen_device.h", CSRC / "jit_device.h", CSRC / "program.hpp",
           CSRC / "jit.hpp", INCLUDE / "mythgpu.h"]
PRELUDE_PARTS = [CSRC / "bv_device.h", CSRC / "keccak_device.h", CSRC / "gen_device.h", CSRC / "jit_device.h"]
PRELUDE_INC = CSRC / "jit_prelude.inc"


def write_prelude() -> None:
    """Embed the device headers the JIT kernels need as one raw string literal
    (hipRTC gets no include path; #include / #pragma once lines are dropped)."""
    body = []
    for p in PRELUDE_PARTS:
        for line in p.read_text().splitlines():
            t = line.strip()
            if t.startswith("#include") or t == "#pragma once":
                continue
            body.append(line)
    text = "R\"MGJ(\n" + "\n".join(body) + "\n)MGJ\"\n"
    if not PRELUDE_INC.exists() or PRELUDE_INC.read_text() != text:
        PRELUDE_INC.write_text(text)

ARCH = os.environ.get("MYTHGPU_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libmythgpu.so)")


def _stale(out: Path, sources) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(p.stat().st_mtime > t for p in list(sources) + HEADERS + [PRELUDE_INC])


def stale() -> bool:
    return _stale(LIB, SOURCES) or _stale(JITD, JITD_SOURCES)


def build_jitd(verbose: bool = False) -> Path:
    """The compiler helper: host code only (comgr is dlopen'ed at run time), so plain g++."""
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        raise RuntimeError("g++ not found (needed for mythgpu_jitd)")
    tmp = JITD.with_suffix(".tmp")
    cmd = [cxx, "-O2", "-std=c++17", "-I/opt/rocm/include", "-o", str(tmp)] + [str(s) for s in JITD_SOURCES] + ["-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"g++ failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(tmp, JITD)
    return JITD


def build(force: bool = False, verbose: bool = False) -> Path:
    write_prelude()
    if force or _stale(JITD, JITD_SOURCES):
        build_jitd(verbose)
    if not force and not _stale(LIB, SOURCES):
        return LIB
    # -structurizecfg-skip-uniform-regions: the interpreter's opcode switch is wave-uniform (an
    # SGPR opcode), so its regions need no exec-mask structurisation; without the option every
    # dispatch walks flow blocks of s_mov/s_andn2/s_cbranch_vccnz (1,879 -> 1,507 SALU in k_run)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-mllvm", "-structurizecfg-skip-uniform-regions",
           "-Wno-unused-result", "-o", str(LIB), "-ldl"] + [str(s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    tmp = LIB.with_suffix(".so.tmp")
    cmd[cmd.index("-o") + 1] = str(tmp)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
