"""ctypes binding of the C restatement (oracle/bveval.c) — test infrastructure
and bench.py's cpu_baseline leg only."""
import ctypes as C

import numpy as np

from oracle.build_c import build

_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(str(build()))
        u32p = C.POINTER(C.c_uint32)
        _lib.bv_search.restype = C.c_int
        _lib.bv_search.argtypes = [u32p, C.c_size_t, u32p, C.c_size_t, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p]
        _lib.bv_eval.restype = C.c_int
        _lib.bv_eval.argtypes = [u32p, C.c_size_t, u32p, C.c_uint64, C.c_void_p]
        _lib.bv_gen_soa.restype = C.c_int
        _lib.bv_gen_soa.argtypes = [u32p, C.c_size_t, u32p, C.c_size_t, C.c_uint64, C.c_uint64, C.c_uint64, u32p]
    return _lib


def _words(blob: bytes) -> np.ndarray:
    return np.frombuffer(blob, dtype=np.uint32).copy()


def search(prog_blob: bytes, gen_blob: np.ndarray, seed: int, start: int, count: int, threads: int = 0,
           verdicts: bool = False):
    p = _words(prog_blob)
    g = np.ascontiguousarray(gen_blob, dtype=np.uint32)
    fh, nh = C.c_uint64(), C.c_uint64()
    ver = np.zeros(count, dtype=np.uint8) if verdicts else None
    rc = lib().bv_search(p.ctypes.data_as(C.POINTER(C.c_uint32)), p.size, g.ctypes.data_as(C.POINTER(C.c_uint32)),
                         g.size, seed, start, count, threads, C.byref(fh), C.byref(nh),
                         ver.ctypes.data if ver is not None else None)
    if rc:
        raise RuntimeError(f"bv_search failed: {rc}")
    first = None if fh.value == (1 << 64) - 1 else fh.value
    return first, nh.value, ver


def eval_soa(prog_blob: bytes, soa: np.ndarray, n: int):
    p = _words(prog_blob)
    soa = np.ascontiguousarray(soa, dtype=np.uint32)
    ver = np.zeros(n, dtype=np.uint8)
    rc = lib().bv_eval(p.ctypes.data_as(C.POINTER(C.c_uint32)), p.size, soa.ctypes.data_as(C.POINTER(C.c_uint32)),
                       n, ver.ctypes.data)
    if rc:
        raise RuntimeError(f"bv_eval failed: {rc}")
    return ver


def gen_soa(prog_blob: bytes, gen_blob: np.ndarray, seed: int, start: int, n: int, coord_words: int) -> np.ndarray:
    """The generated coordinates of candidates [start, start+n) as SoA rows (mg_eval layout)."""
    p = _words(prog_blob)
    g = np.ascontiguousarray(gen_blob, dtype=np.uint32)
    soa = np.zeros((max(coord_words, 1), n), dtype=np.uint32)
    u32p = C.POINTER(C.c_uint32)
    rc = lib().bv_gen_soa(p.ctypes.data_as(u32p), p.size, g.ctypes.data_as(u32p), g.size, seed, start, n,
                          soa.ctypes.data_as(u32p))
    if rc:
        raise RuntimeError(f"bv_gen_soa failed: {rc}")
    return soa
