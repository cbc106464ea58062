"""ctypes binding of ``libmythgpu.so`` (C-ABI in ``include/mythgpu.h``).

The reference reaches its solver through z3py's ctypes binding of libz3; this
module is the same kind of binding for the GPU engine.  There is no CPU
fallback: if the library or a gfx950 device is missing, the calls raise
:class:`EngineError` (the ``get_model`` hook then leaves the query to z3).
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import threading
from pathlib import Path
from typing import Optional

import numpy as np

LIB_PATH = Path(__file__).resolve().parent / "libmythgpu.so"

MG_OK = 0
MG_E_INVALID = -1
MG_E_UNSUPPORTED = -2
MG_E_HIP = -3
MG_E_NODEVICE = -4
MG_E_NOMEM = -5
MG_E_NOTINIT = -6
MG_SEARCH_EARLY_EXIT = 1
MG_JIT_GEN_VERDICTS = 1
MG_JIT_ASM = 2  # the first tier: gfx950 assembly emitted by the engine (jit_asm.cpp)
MG_JIT_SOA_TILED = 4  # eval kernels read the tiled SoA (tile_soa)
MG_JIT_O3 = 8  # the O3 eval kernel even with watch rows (the first tier's is the default there)


def tile_soa(soa):
    """[row][candidate] SoA (rows x n, numpy or torch) -> the tiled layout MG_JIT_SOA_TILED kernels
    read: word ((i // 64) * rows + r) * 64 + i % 64 (the last 64-candidate block zero-padded)."""
    rows, n = soa.shape
    blocks = (n + 63) // 64
    pad = blocks * 64 - n
    if hasattr(soa, "permute"):  # torch
        import torch

        x = torch.nn.functional.pad(soa, (0, pad)) if pad else soa
        return x.reshape(rows, blocks, 64).permute(1, 0, 2).contiguous()
    x = np.pad(soa, ((0, 0), (0, pad))) if pad else soa
    return np.ascontiguousarray(x.reshape(rows, blocks, 64).transpose(1, 0, 2))
NO_HIT = (1 << 64) - 1

EXPORTS = [
    "mg_init", "mg_collective_kind", "mg_shutdown", "mg_last_error", "mg_version", "mg_program_check", "mg_program_check_gen",
    "mg_program_specialized", "mg_program_load",
    "mg_program_info", "mg_program_free", "mg_gen_load", "mg_gen_info", "mg_gen_free", "mg_eval", "mg_eval_dev",
    "mg_eval_generated", "mg_search", "mg_keccak256", "mg_stats", "mg_stats_reset", "mg_dev_alloc",
    "mg_dev_free", "mg_dev_upload", "mg_dev_download", "mg_program_jit_source", "mg_program_jit_asm", "mg_code_object_check", "mg_jit_compile", "mg_jit_compile_ex", "mg_jit_verdicts", "mg_jit_info", "mg_jit_layout",
    "mg_jit_compile_async", "mg_jit_poll", "mg_jit_cancel", "mg_jit_helper_pid", "mg_cache_clear", "mg_split_range",
    "mg_jit_free", "mg_jit_search", "mg_jit_search_many", "mg_jit_eval", "mg_jit_eval_dev",
]


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mythgpu error {code}: {msg}")
        self.code = code


class EngineUnsupported(EngineError):
    pass


class ProgramInfo(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32), ("n_instrs", C.c_uint32), ("n_coords", C.c_uint32), ("n_roots", C.c_uint32),
        ("value_words", C.c_uint32), ("uses_lds", C.c_uint32), ("n_watch", C.c_uint32),
        ("watch_words", C.c_uint32), ("coord_words", C.c_uint32), ("reserved", C.c_uint32),
        ("limb_ops", C.c_uint64),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("programs_loaded", C.c_uint64), ("launches", C.c_uint64), ("candidates", C.c_uint64),
        ("hits", C.c_uint64), ("kernel_ms_total", C.c_double), ("last_kernel_ms", C.c_double),
        ("last_candidates", C.c_uint64), ("device", C.c_uint32), ("cu_count", C.c_uint32),
        ("clock_mhz", C.c_uint32), ("n_devices", C.c_uint32), ("jit_refused", C.c_uint64),
    ]


_lib = None
_lib_lock = threading.Lock()


def _shutdown_at_exit():
    lib = _lib
    if lib is not None:
        try:
            lib.mg_shutdown()
        except Exception:  # exiting anyway
            pass


def load_library(path: Optional[Path] = None) -> C.CDLL:
    """Load (and type) the shared library.  Loading needs no GPU."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        p = Path(path or LIB_PATH)
        if not p.exists():
            raise EngineError(MG_E_NODEVICE, f"{p} is not built (run mythril_amd.build.build())")
        lib = C.CDLL(str(p))
        u8p, u32p, u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
        sig = {
            "mg_init": (C.c_int, [C.c_uint32]),
            "mg_collective_kind": (C.c_int, []),
            "mg_shutdown": (None, []),
            "mg_last_error": (C.c_char_p, []),
            "mg_version": (C.c_int, []),
            "mg_program_check": (C.c_int, [u8p, C.c_size_t, C.POINTER(ProgramInfo)]),
            "mg_program_check_gen": (C.c_int, [u8p, C.c_size_t, u32p, C.c_size_t, C.POINTER(ProgramInfo)]),
            "mg_program_specialized": (C.c_int, [u8p, C.c_size_t, u32p, C.c_size_t, C.c_uint32, u32p, C.c_size_t,
                                                 C.POINTER(C.c_size_t)]),
            "mg_program_load": (C.c_int, [u8p, C.c_size_t, u64p]),
            "mg_program_info": (C.c_int, [C.c_uint64, C.POINTER(ProgramInfo)]),
            "mg_program_free": (C.c_int, [C.c_uint64]),
            "mg_gen_load": (C.c_int, [C.c_uint64, u32p, C.c_size_t, u64p]),
            "mg_gen_info": (C.c_int, [C.c_uint64, C.POINTER(ProgramInfo)]),
            "mg_gen_free": (C.c_int, [C.c_uint64]),
            "mg_eval": (C.c_int, [C.c_uint64, u32p, C.c_uint64, u8p, u32p]),
            "mg_eval_dev": (C.c_int, [C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
            "mg_eval_generated": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, u8p, u32p]),
            "mg_search": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                    u64p, u64p, u32p]),
            "mg_keccak256": (C.c_int, [u8p, u32p, C.c_uint64, u8p]),
            "mg_stats": (C.c_int, [C.POINTER(Stats)]),
            "mg_stats_reset": (C.c_int, []),
            "mg_dev_alloc": (C.c_int, [C.c_size_t, C.POINTER(C.c_void_p)]),
            "mg_dev_free": (C.c_int, [C.c_void_p]),
            "mg_dev_upload": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
            "mg_dev_download": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
            "mg_program_jit_source": (C.c_int, [u8p, C.c_size_t, u32p, C.c_size_t, C.c_int, C.c_char_p,
                                                C.c_size_t, C.POINTER(C.c_size_t)]),
            "mg_code_object_check": (C.c_int, [C.c_void_p, C.c_size_t, u32p, u32p, u32p, u32p]),
            "mg_program_jit_asm": (C.c_int, [u8p, C.c_size_t, u32p, C.c_size_t, C.c_int, C.c_char_p,
                                             C.c_size_t, C.POINTER(C.c_size_t)]),
            "mg_jit_compile": (C.c_int, [C.c_uint64, C.c_uint64, u64p]),
            "mg_jit_compile_ex": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint32, u64p]),
            "mg_jit_verdicts": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, u8p]),
            "mg_jit_info": (C.c_int, [C.c_uint64, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
            "mg_jit_layout": (C.c_int, [C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
            "mg_jit_compile_async": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint32, u64p]),
            "mg_jit_poll": (C.c_int, [C.c_uint64, C.c_int32, u64p]),
            "mg_jit_cancel": (C.c_int, [C.c_uint64]),
            "mg_jit_helper_pid": (C.c_int, []),
            "mg_cache_clear": (C.c_int, []),
            "mg_split_range": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint32, u64p, u64p]),
            "mg_jit_free": (C.c_int, [C.c_uint64]),
            "mg_jit_search": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, u64p, u64p, u32p]),
            "mg_jit_search_many": (C.c_int, [C.c_uint64, C.c_uint32, u64p, u64p, u64p, C.c_uint32, u64p, u64p]),
            "mg_jit_eval": (C.c_int, [C.c_uint64, u32p, C.c_uint64, u8p, u32p]),
            "mg_jit_eval_dev": (C.c_int, [C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        # stop the engine (its compile thread finishes any compile in flight, modules and
        # device buffers are released) while Python is still finalising, i.e. before the
        # C-level exit handlers and library destructors run: a compile thread still inside the
        # compiler, or HIP work, racing the runtime's teardown can crash the process at exit
        atexit.register(_shutdown_at_exit)
        return lib


def jit_helper_pid() -> int:
    """pid of the compiler helper process (-1: not started yet, -2: it died; JIT off)."""
    return int(load_library().mg_jit_helper_pid())


def _check(rc: int):
    if rc != MG_OK:
        msg = (_lib.mg_last_error() or b"").decode(errors="replace")
        if rc == MG_E_UNSUPPORTED:
            raise EngineUnsupported(rc, msg)
        raise EngineError(rc, msg)


def _u8(buf: bytes):
    arr = (C.c_uint8 * len(buf)).from_buffer_copy(buf)
    return arr


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def check_program(blob: bytes) -> ProgramInfo:
    """Validate + lower a program on the host (no GPU)."""
    lib = load_library()
    info = ProgramInfo()
    _check(lib.mg_program_check(_u8(blob), len(blob), C.byref(info)))
    return info


def check_program_gen(blob: bytes, gen_blob: np.ndarray) -> ProgramInfo:
    """Host-only: the program specialised for a generator (what a search runs)."""
    lib = load_library()
    g = np.ascontiguousarray(gen_blob, dtype=np.uint32)
    info = ProgramInfo()
    _check(lib.mg_program_check_gen(_u8(blob), len(blob), _ptr(g, C.c_uint32), g.size, C.byref(info)))
    return info


MG_SPEC_MAGIC = 0x43455053
MG_SPEC_KEEP_WATCH = 1
MG_SPEC_INTERP = 2


def specialized_program(blob: bytes, gen_blob: Optional[np.ndarray] = None, keep_watch: bool = False,
                        interp: bool = False) -> dict:
    """Host-only ``mg_program_specialized``: the lowered, specialised program a search (with a
    generator) or an eval (without) runs, in SSA form — ``code`` (n x 8 uint32:
    op, width, dst, a, b, c, p0, p1), ``consts``, ``aux``, ``widths``, ``n_coords``.  ``interp``:
    the interpreter's program (literal-tail keys narrowed) instead of the compiled kernel's."""
    lib = load_library()
    g = None if gen_blob is None else np.ascontiguousarray(gen_blob, dtype=np.uint32)
    gp = _ptr(g, C.c_uint32) if g is not None else None
    gn = 0 if g is None else g.size
    flags = (MG_SPEC_KEEP_WATCH if keep_watch else 0) | (MG_SPEC_INTERP if interp else 0)
    n = C.c_size_t()
    _check(lib.mg_program_specialized(_u8(blob), len(blob), gp, gn, flags, None, 0, C.byref(n)))
    w = np.zeros(n.value, dtype=np.uint32)
    _check(lib.mg_program_specialized(_u8(blob), len(blob), gp, gn, flags, _ptr(w, C.c_uint32), w.size,
                                      C.byref(n)))
    assert int(w[0]) == MG_SPEC_MAGIC
    ni, nc, na, nv, ncoord = (int(x) for x in w[1:6])
    pos = 6
    code = w[pos:pos + 8 * ni].reshape(ni, 8)
    pos += 8 * ni
    consts = w[pos:pos + nc]
    pos += nc
    aux = w[pos:pos + na]
    pos += na
    widths = w[pos:pos + nv]
    return {"code": code, "consts": consts, "aux": aux, "widths": widths, "n_coords": ncoord}


def jit_source(blob: bytes, gen_blob: Optional[np.ndarray] = None, compile: bool = False, tiled: bool = False) -> str:
    """Host-only: the specialised HIP source of a program — the search kernel when a
    generator blob is given, else the eval kernel — optionally hipRTC-compiled (no GPU)."""
    lib = load_library()
    g = None if gen_blob is None else np.ascontiguousarray(gen_blob, dtype=np.uint32)
    gp = _ptr(g, C.c_uint32) if g is not None else None
    gn = 0 if g is None else g.size
    n = C.c_size_t()
    _check(lib.mg_program_jit_source(_u8(blob), len(blob), gp, gn, 2 if tiled else 0, None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value + 1)
    _check(lib.mg_program_jit_source(_u8(blob), len(blob), gp, gn, (1 if compile else 0) | (2 if tiled else 0), buf,
                                     n.value + 1, C.byref(n)))
    return buf.value.decode()


def jit_asm(blob: bytes, gen_blob: Optional[np.ndarray] = None, compile: bool = False, tiled: bool = False) -> str:
    """Host-only: the first tier's gfx950 assembly — of a search program (mgj_search + mgj_gen)
    when a generator blob is given, else of the eval kernel (mgj_eval) — optionally assembled and
    linked through comgr (no GPU).  Raises EngineUnsupported for programs outside the tier."""
    lib = load_library()
    g = None if gen_blob is None else np.ascontiguousarray(gen_blob, dtype=np.uint32)
    gp = _ptr(g, C.c_uint32) if g is not None else None
    gn = 0 if g is None else g.size
    n = C.c_size_t()
    _check(lib.mg_program_jit_asm(_u8(blob), len(blob), gp, gn, 2 if tiled else 0, None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value + 1)
    _check(lib.mg_program_jit_asm(_u8(blob), len(blob), gp, gn, (1 if compile else 0) | (2 if tiled else 0), buf,
                                  n.value + 1, C.byref(n)))
    return buf.value.decode()


def split_range(start: int, count: int, n_dev: int):
    """Host-only ``mg_split_range``: the [start, start+count) slice each of ``n_dev`` devices
    sweeps in a multi-device ``mg_search`` — [(start_d, count_d)] in device order."""
    lib = load_library()
    st = (C.c_uint64 * max(n_dev, 1))()
    ct = (C.c_uint64 * max(n_dev, 1))()
    _check(lib.mg_split_range(start, count, n_dev, st, ct))
    return [(st[i], ct[i]) for i in range(n_dev)]


def device_mask_from_env() -> int:
    """``MYTHGPU_DEVICES``: "all" or a comma list of GPU indices opens several GPUs in this
    process (the shim splits every search over them); otherwise one GPU,
    ``MYTHGPU_DEVICE`` / ``LOCAL_RANK`` (one process per GPU, the torch.distributed layout)."""
    spec = os.environ.get("MYTHGPU_DEVICES")
    if spec:
        if spec.strip() == "all":
            return 0xFFFFFFFF
        return sum(1 << int(x) for x in spec.split(",") if x.strip())
    return 1 << int(os.environ.get("MYTHGPU_DEVICE", os.environ.get("LOCAL_RANK", "0")))


class Engine:
    """Process-wide handle on the engine: one GPU (one process per GPU), or every GPU of
    ``MYTHGPU_DEVICES`` with searches split across them inside the shim."""

    _instance = None
    _ilock = threading.Lock()

    @classmethod
    def get(cls) -> "Engine":
        with cls._ilock:
            if cls._instance is None:
                cls._instance = Engine()
            return cls._instance

    def __init__(self, device: Optional[int] = None, mask: Optional[int] = None):
        self.lib = load_library()
        if mask is None:
            mask = (1 << device) if device is not None else device_mask_from_env()
        _check(self.lib.mg_init(mask))
        self.mask = mask
        self.device = (mask & -mask).bit_length() - 1 if mask else 0

    def reinit(self, mask: int) -> None:
        """Shut the engine down (every handle becomes invalid) and open ``mask`` instead."""
        self.lib.mg_shutdown()
        _check(self.lib.mg_init(mask))
        self.mask = mask

    @property
    def n_devices(self) -> int:
        return self.stats().n_devices

    # programs -------------------------------------------------------
    def load(self, blob: bytes) -> int:
        h = C.c_uint64()
        _check(self.lib.mg_program_load(_u8(blob), len(blob), C.byref(h)))
        return h.value

    def info(self, prog: int) -> ProgramInfo:
        info = ProgramInfo()
        _check(self.lib.mg_program_info(prog, C.byref(info)))
        return info

    def free(self, prog: int):
        _check(self.lib.mg_program_free(prog))

    def load_gen(self, prog: int, blob: np.ndarray) -> int:
        blob = np.ascontiguousarray(blob, dtype=np.uint32)
        h = C.c_uint64()
        _check(self.lib.mg_gen_load(prog, _ptr(blob, C.c_uint32), blob.size, C.byref(h)))
        return h.value

    def gen_info(self, gen: int) -> ProgramInfo:
        """The generator-specialised program the searches run."""
        info = ProgramInfo()
        _check(self.lib.mg_gen_info(gen, C.byref(info)))
        return info

    def free_gen(self, gen: int):
        _check(self.lib.mg_gen_free(gen))

    # evaluation -----------------------------------------------------
    def eval(self, prog: int, soa: np.ndarray, n: int, watch_words: int = 0):
        """Evaluate n candidates given as a [coord_words][n] uint32 SoA."""
        soa = np.ascontiguousarray(soa, dtype=np.uint32)
        info = self.info(prog)  # mg_eval reads coord_words x n words and writes watch_words x n
        if soa.size < info.coord_words * n:
            raise ValueError(f"eval: SoA of {soa.size} words, the program reads {info.coord_words} x {n}")
        if watch_words and watch_words < info.watch_words:
            raise ValueError(f"eval: program stores {info.watch_words} watch rows, caller asked for {watch_words}")
        ver = np.zeros(n, dtype=np.uint8)
        watch = np.zeros((max(watch_words, 1), n), dtype=np.uint32) if watch_words else None
        _check(self.lib.mg_eval(prog, _ptr(soa, C.c_uint32), n, _ptr(ver, C.c_uint8),
                                _ptr(watch, C.c_uint32) if watch is not None else None))
        return ver, watch

    def eval_generated(self, prog: int, gen: int, seed: int, start: int, n: int, watch_words: int = 0):
        ver = np.zeros(n, dtype=np.uint8)
        watch = np.zeros((max(watch_words, 1), n), dtype=np.uint32) if watch_words else None
        _check(self.lib.mg_eval_generated(prog, gen, seed, start, n, _ptr(ver, C.c_uint8),
                                          _ptr(watch, C.c_uint32) if watch is not None else None))
        return ver, watch

    def search(self, prog: int, gen: int, seed: int, start: int, count: int, early_exit: bool = True,
               assign: Optional[np.ndarray] = None):
        """(first hit or None, hit count); with ``assign`` (uint32[watch_words]) the winning
        candidate's watch rows are written into it."""
        fh, nh = C.c_uint64(), C.c_uint64()
        flags = MG_SEARCH_EARLY_EXIT if early_exit else 0
        ap = _ptr(assign, C.c_uint32) if assign is not None else None
        _check(self.lib.mg_search(prog, gen, seed, start, count, flags, C.byref(fh), C.byref(nh), ap))
        return (None if fh.value == NO_HIT else fh.value), nh.value

    # JIT-specialised kernels --------------------------------------
    def jit_compile(self, prog: int, gen: int = 0, gen_verdicts: bool = False, asm: bool = False,
                    tiled: bool = False, o3: bool = False) -> int:
        """``asm``: the first tier (assembly emitted by the engine).  ``tiled`` (eval kernels): the
        kernel reads the tiled SoA (:func:`tile_soa`; MG_JIT_SOA_TILED in mythgpu.h).  An eval kernel
        with watch rows is the first tier's unless ``o3`` (MG_JIT_O3)."""
        h = C.c_uint64()
        flags = (MG_JIT_GEN_VERDICTS if gen_verdicts else 0) | (MG_JIT_ASM if asm else 0) | \
            (MG_JIT_SOA_TILED if tiled else 0) | (MG_JIT_O3 if o3 else 0)
        _check(self.lib.mg_jit_compile_ex(prog, gen, flags, C.byref(h)))
        return h.value

    def jit_compile_async(self, prog: int, gen: int = 0, gen_verdicts: bool = False, asm: bool = False) -> int:
        """Start compiling on the engine's compile thread; returns a ticket for :meth:`jit_poll`."""
        t = C.c_uint64()
        flags = (MG_JIT_GEN_VERDICTS if gen_verdicts else 0) | (MG_JIT_ASM if asm else 0)
        _check(self.lib.mg_jit_compile_async(prog, gen, flags, C.byref(t)))
        return t.value

    def jit_poll(self, ticket: int, wait_ms: int = 0) -> Optional[int]:
        """The JIT handle once the compile is done (the ticket is then consumed), else None.
        A failed compile raises (and consumes the ticket)."""
        h = C.c_uint64()
        _check(self.lib.mg_jit_poll(ticket, wait_ms, C.byref(h)))
        return h.value or None

    def jit_cancel(self, ticket: int) -> None:
        _check(self.lib.mg_jit_cancel(ticket))

    def cache_clear(self) -> None:
        """Drop the engine's host-side caches (cold-start measurements)."""
        _check(self.lib.mg_cache_clear())

    def jit_verdicts(self, jit: int, seed: int, start: int, n: int) -> np.ndarray:
        """Per-candidate verdicts of the JIT kernel (compiled with ``gen_verdicts``)."""
        ver = np.zeros(n, dtype=np.uint8)
        _check(self.lib.mg_jit_verdicts(jit, seed, start, n, _ptr(ver, C.c_uint8)))
        return ver

    def jit_info(self, jit: int):
        ms, nb = C.c_double(), C.c_int()
        _check(self.lib.mg_jit_info(jit, C.byref(ms), C.byref(nb)))
        return ms.value, nb.value

    def jit_layout(self, jit: int):
        """(flags, coord_words, watch_words) of a JIT handle (mg_jit_layout): flags has MG_JIT_ASM for the
        first tier's kernels, MG_JIT_SOA_TILED for an eval kernel that reads the tiled SoA."""
        f, cw, ww = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _check(self.lib.mg_jit_layout(jit, C.byref(f), C.byref(cw), C.byref(ww)))
        return f.value, cw.value, ww.value

    def jit_free(self, jit: int):
        _check(self.lib.mg_jit_free(jit))

    def jit_search(self, jit: int, seed: int, start: int, count: int, early_exit: bool = True,
                   assign: Optional[np.ndarray] = None):
        fh, nh = C.c_uint64(), C.c_uint64()
        flags = MG_SEARCH_EARLY_EXIT if early_exit else 0
        ap = _ptr(assign, C.c_uint32) if assign is not None else None
        _check(self.lib.mg_jit_search(jit, seed, start, count, flags, C.byref(fh), C.byref(nh), ap))
        return (None if fh.value == NO_HIT else fh.value), nh.value

    def jit_search_many(self, jit: int, seeds, starts, counts, early_exit: bool = False):
        """Independent searches (seed, start, count) of one kernel in one call (mg_jit_search_many):
        [(first_hit or None, hits)] in order."""
        n = len(seeds)
        s = np.ascontiguousarray(seeds, dtype=np.uint64)
        a = np.ascontiguousarray(starts, dtype=np.uint64)
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        if not (len(a) == len(c) == n):
            raise ValueError("seeds, starts and counts differ in length")
        fh = np.zeros(n, dtype=np.uint64)
        nh = np.zeros(n, dtype=np.uint64)
        flags = MG_SEARCH_EARLY_EXIT if early_exit else 0
        _check(self.lib.mg_jit_search_many(jit, n, _ptr(s, C.c_uint64), _ptr(a, C.c_uint64), _ptr(c, C.c_uint64),
                                           flags, _ptr(fh, C.c_uint64), _ptr(nh, C.c_uint64)))
        return [(None if int(f) == NO_HIT else int(f), int(h)) for f, h in zip(fh, nh)]

    def jit_eval(self, jit: int, soa: np.ndarray, n: int, watch_words: int = 0):
        """Verdicts (and watch rows) of n explicit candidates.  The SoA is checked against the kernel's
        layout first: [coord_words][n] row-major, or tile_soa's (blocks, coord_words, 64) for a kernel
        compiled ``tiled`` — mg_jit_eval copies coord_words x n (tiled: x ceil(n/64) x 64) words from it."""
        flags, cw, ww = self.jit_layout(jit)
        # mg_jit_eval copies the kernel's own watch_words rows into watch_out: a buffer sized from a
        # smaller count would be overrun
        if watch_words and watch_words < ww:
            raise ValueError(f"eval kernel stores {ww} watch rows, caller asked for {watch_words}")
        if flags & MG_JIT_SOA_TILED:
            blocks = (n + 63) // 64
            if getattr(soa, "ndim", 0) != 3 or tuple(soa.shape[1:]) != (cw, 64) or soa.shape[0] < blocks:
                raise ValueError(f"tiled eval kernel: expected the tiled SoA ({blocks}, {cw}, 64) of tile_soa, "
                                 f"got shape {getattr(soa, 'shape', None)}")
        elif cw and (getattr(soa, "ndim", 0) != 2 or soa.shape[0] != cw or soa.shape[1] < n):
            raise ValueError(f"eval kernel: expected the [row][candidate] SoA ({cw}, {n}), got shape "
                             f"{getattr(soa, 'shape', None)}")
        soa = np.ascontiguousarray(soa, dtype=np.uint32)
        if soa.shape[-1] != n and not (flags & MG_JIT_SOA_TILED):
            soa = np.ascontiguousarray(soa[:, :n])
        ver = np.zeros(n, dtype=np.uint8)
        watch = np.zeros((max(watch_words, 1), n), dtype=np.uint32) if watch_words else None
        _check(self.lib.mg_jit_eval(jit, _ptr(soa, C.c_uint32), n, _ptr(ver, C.c_uint8),
                                    _ptr(watch, C.c_uint32) if watch is not None else None))
        return ver, watch

    def keccak256(self, msgs):
        msgs = [bytes(m) for m in msgs]
        n = len(msgs)
        if n == 0:
            return []
        cat = b"".join(msgs) or b"\0"
        lens = np.array([len(m) for m in msgs], dtype=np.uint32)
        out = np.zeros(n * 32, dtype=np.uint8)
        _check(self.lib.mg_keccak256(_u8(cat), _ptr(lens, C.c_uint32), n, _ptr(out, C.c_uint8)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(n)]

    def stats(self) -> Stats:
        s = Stats()
        _check(self.lib.mg_stats(C.byref(s)))
        return s

    def reset_stats(self):
        _check(self.lib.mg_stats_reset())

    # device buffers (inputs resident in HBM) ------------------------
    def dev_alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        _check(self.lib.mg_dev_alloc(nbytes, C.byref(p)))
        return p.value

    def dev_free(self, p: int):
        _check(self.lib.mg_dev_free(p))

    def dev_upload(self, p: int, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        _check(self.lib.mg_dev_upload(p, arr.ctypes.data, arr.nbytes))

    def dev_download(self, arr: np.ndarray, p: int):
        _check(self.lib.mg_dev_download(arr.ctypes.data, p, arr.nbytes))

    def eval_dev(self, prog: int, d_soa: int, n: int, d_ver: int, d_watch: int = 0):
        _check(self.lib.mg_eval_dev(prog, d_soa, n, d_ver, d_watch or None))

    def jit_eval_dev(self, jit: int, d_soa: int, n: int, d_ver: int, d_watch: int = 0):
        """The compiled eval kernel on HBM-resident SoA inputs (device pointers)."""
        _check(self.lib.mg_jit_eval_dev(jit, d_soa, n, d_ver, d_watch or None))
