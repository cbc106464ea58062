"""The identities the round-6 generator rewrites rest on, checked exhaustively or over large random
samples on the CPU (the GPU tests then compare the rewritten kernels with the C port per candidate):

* the folded key (jit_asm.cpp ``grnd``, gen_device.h ``GKeys.kf``): gfin's first xor-shift is linear,
  ``(k ^ s) ^ ((k ^ s) >> 16) == (k ^ (k >> 16)) ^ (s ^ (s >> 16))``;
* the one-multiply dictionary index (``dict_index``): for ``n < 256`` and ``a = h >> 16``,
  ``(a * n) >> 16`` is the high word of the 24-bit product ``a * (n << 16)`` (``v_mul_hi_u32_u24``);
* the one-instruction ALIGNED offset: ``base + (m << sh)`` over two limbs, ``sh <= 6``, equals
  ``m * 2**sh + base`` modulo 2**64 (``v_mad_u64_u32``) when the sum fits the two limbs the carry
  can reach.

Reference anchor: the GEN3 candidate stream these draws define (``include/mythgpu.h`` GEN3 comment,
``oracle/bveval.c`` gen_value) — the verdicts of ``Model.eval`` (``mythril/laser/smt/model.py:45-59``)
over it are what the kernels report."""
import numpy as np


def test_key_fold_is_exact():
    rng = np.random.default_rng(6)
    k = rng.integers(0, 1 << 32, size=1 << 20, dtype=np.uint64).astype(np.uint32)
    s = rng.integers(0, 1 << 32, size=1 << 20, dtype=np.uint64).astype(np.uint32)
    x = k ^ s
    assert np.array_equal(x ^ (x >> np.uint32(16)), (k ^ (k >> np.uint32(16))) ^ (s ^ (s >> np.uint32(16))))


def test_mulhi24_index_is_exact():
    a = np.arange(1 << 16, dtype=np.uint64)
    for n in range(1, 256):
        want = (a * np.uint64(n)) >> np.uint64(16)
        p = (a & np.uint64(0xFFFFFF)) * (np.uint64(n << 16) & np.uint64(0xFFFFFF))  # the 24-bit operands
        got = p >> np.uint64(32)
        assert np.array_equal(want, got), n
        assert int(want.max()) < n


def test_aligned_mad_is_exact():
    rng = np.random.default_rng(7)
    m = rng.integers(0, 1 << 32, size=1 << 18, dtype=np.uint64)
    for sh in range(1, 7):
        base = int(rng.integers(0, 1 << 62))
        lo, hi = base & 0xFFFFFFFF, base >> 32
        # the shift-and-carry form: limb 0 = lo + (m << sh mod 2^32), limb 1 = hi + (m >> (32 - sh)) + carry
        s0 = (m << np.uint64(sh)) & np.uint64(0xFFFFFFFF)
        s1 = m >> np.uint64(32 - sh)
        l0 = (s0 + np.uint64(lo)) & np.uint64(0xFFFFFFFF)
        carry = ((s0 + np.uint64(lo)) >> np.uint64(32)) & np.uint64(1)
        l1 = (s1 + np.uint64(hi) + carry) & np.uint64(0xFFFFFFFF)
        mad = (m * np.uint64(1 << sh) + np.uint64(base)) & np.uint64((1 << 64) - 1)
        assert np.array_equal(l0, mad & np.uint64(0xFFFFFFFF)), sh
        assert np.array_equal(l1, mad >> np.uint64(32)), sh
