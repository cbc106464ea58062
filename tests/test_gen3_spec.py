"""GEN3 candidate generator: the formulas documented in include/mythgpu.h, restated here in
Python, against the C restatement (oracle/bveval.c) — and, with -m gpu, against both GPU
kernels (interpreter and JIT).  A one-constraint program ``x == v`` holds at index i exactly
when the generator gives x the value v there, so each check reads the generator through the
same search entry points the product uses.  (Test-side restatement; no reference file holds
the generator: it is this engine's own candidate stream)"""
import random

import pytest

from mythril_amd import search, ssa
from mythril_amd.smt import symbol_factory
from oracle import cport

M32, M64 = (1 << 32) - 1, (1 << 64) - 1


def fmix64(x):
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & M64
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & M64
    x ^= x >> 33
    return x


def keys(idx, seed):
    G = fmix64((idx >> 6) ^ fmix64(seed ^ 0xBB67AE8584CAA73B))
    K = G ^ fmix64((idx & 63) ^ fmix64(seed ^ 0x6A09E667F3BCC908))
    return K & M32, K >> 32, G & M32, G >> 32


def salt(c, j):
    return (c * 0x9E3779B9 + j * 0x85EBCA6B + 0x27D4EB2F) & M32


def fin(x):
    x ^= x >> 16
    x = ((x & 0xFFFFFF) * 0x9E3779) & M32
    x ^= x >> 15
    return x


def rnd(k, c, j):
    return (fin(k[0] ^ salt(c, j)) + k[1]) & M32


def wsel(k, c):
    return ((k[2] ^ salt(c, 0xFFFE)) * 0x9E3779B1 + k[3]) & M32


def uniform_raw(k, c, L):
    u = []
    for j in range(L):
        if j < 2:
            u.append(rnd(k, c, j))
        else:
            s = (7 * j + 3) % 31 + 1
            u.append(((((u[j - 1] << 32) | u[j - 2]) >> s) + u[j - 2]) & M32)
    return u


def value(limbs, w):
    return sum(x << (32 * j) for j, x in enumerate(limbs)) & ((1 << w) - 1)


def one_query(w, v, spec):
    """(program blob, generator blob) of ``x == v`` with x's generator set by ``spec(gb, c)``."""
    x = symbol_factory.BitVecSym("g3x", w)
    P = ssa.flatten([(x == symbol_factory.BitVecVal(v, w)).raw])
    (c,) = [co.index for co in P.coords if co.name == "g3x"]
    gb = search.GenBuilder(P)
    spec(gb, c)
    return P.to_bytes(), gb.blob(), c


def hits(prog, gen, seed, idx):
    first, n, _ = cport.search(prog, gen, seed, idx, 1)
    return first == idx and n == 1


SEED = 0x6D797468
rng = random.Random(3)
# indices whose low 32-bit word has bit 31 set pin the kernels' 64-bit index handling (a
# sign-extended readfirstlane once corrupted the high word of such group bases in the JIT)
INDICES = [0, 1, 63, 64, 65, (1 << 31) + 7, (1 << 40) | 0x80000041, 1 << 20, (1 << 40) + 17, (1 << 63) + 5,
           (1 << 63) | 0xFFFFFFC3] + [rng.getrandbits(64) for _ in range(6)]


@pytest.mark.parametrize("w", [256, 160, 64, 33, 32, 20])
def test_uniform_matches_documented_formula(w):
    L = (w + 31) // 32
    for idx in INDICES:
        # the coordinate index is known only after flattening: flatten once to learn it
        _, _, c = one_query(w, 0, lambda gb, c: gb.uniform(c))
        want = value(uniform_raw(keys(idx, SEED), c, L), w)
        prog, gen, _ = one_query(w, want, lambda gb, c: gb.uniform(c))
        assert hits(prog, gen, SEED, idx), (w, idx)
        prog, gen, _ = one_query(w, want ^ 1, lambda gb, c: gb.uniform(c))
        assert not hits(prog, gen, SEED, idx), (w, idx)


def test_dict_and_mixed_choice_match_documented_formula():
    w, vals = 256, [5, 1 << 200, (1 << 256) - 1]
    _, _, c = one_query(w, 0, lambda gb, c: gb.dict(c, vals))
    for idx in INDICES:
        k = keys(idx, SEED)
        e = ((rnd(k, c, 0xFFFF) >> 16) * len(vals)) >> 16
        prog, gen, _ = one_query(w, vals[e], lambda gb, c: gb.dict(c, vals))
        assert hits(prog, gen, SEED, idx)
        # MIXED, DICT with probability 1/2 else SMALL (8 bits): the group word picks the branch
        spec = lambda gb, c: gb.mixed(c, vals, p_dict=0.5, small_bits=8, p_small=0.5)  # noqa: E731
        pd = int(0.5 * 65536)
        if (wsel(k, c) >> 16) < pd:
            want = vals[e]
        else:
            want = uniform_raw(k, c, 1)[0] & 0xFF
        prog, gen, _ = one_query(w, want, spec)
        assert hits(prog, gen, SEED, idx), idx


@pytest.mark.gpu
def test_gpu_kernels_follow_documented_formula():
    from mythril_amd import native

    eng = native.Engine.get()
    w = 256
    _, _, c = one_query(w, 0, lambda gb, c: gb.uniform(c))
    for idx in INDICES[:11]:
        want = value(uniform_raw(keys(idx, SEED), c, 8), w)
        prog_b, gen_b, _ = one_query(w, want, lambda gb, c: gb.uniform(c))
        prog = eng.load(prog_b)
        gh = eng.load_gen(prog, gen_b)
        try:
            assert eng.search(prog, gh, SEED, idx, 1, early_exit=False) == (idx, 1)
            jh = eng.jit_compile(prog, gh)
            try:
                assert eng.jit_search(jh, SEED, idx, 1, early_exit=False) == (idx, 1)
            finally:
                eng.jit_free(jh)
        finally:
            eng.free_gen(gh)
            eng.free(prog)
