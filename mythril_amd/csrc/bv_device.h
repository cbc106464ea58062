// 256-bit (8 x 32-bit limb) bit-vector arithmetic in VGPRs for gfx950.
//
// All arrays are indexed with compile-time constants only (fully unrolled
// loops), so they stay in registers: a runtime-indexed private array is
// demoted to scratch on AMDGPU.  Per-lane data-dependent amounts (shift
// counts, exponent bits) are handled with barrel stages and predication, never
// with runtime register indexing.
//
// Semantics follow SMT-LIB QF_BV (what z3 evaluates for LASER's terms,
// SURVEY.md §2.3): total division (x/0 = ~0, x%0 = x), shifts >= w saturate.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mg {

typedef uint32_t u32;
typedef uint64_t u64;

struct W8 {
  u32 w[8];
};

__device__ __forceinline__ u32 top_mask(u32 width) {
  u32 r = width & 31u;
  return r ? ((1u << r) - 1u) : 0xFFFFFFFFu;
}

// mask limbs above `width` (width <= 256) to zero
__device__ __forceinline__ void canon8(W8& x, u32 width) {
  const u32 L = (width + 31u) >> 5;
  const u32 tm = top_mask(width);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u32 v = x.w[i];
    v = (u32)i < L ? v : 0u;
    v = (u32)i == L - 1 ? (v & tm) : v;
    x.w[i] = v;
  }
}

// carry / borrow chains through __builtin_addc/__builtin_subc: one v_add_co/v_addc_co
// (v_sub_co/v_subb_co) per limb, no 64-bit temporaries
__device__ __forceinline__ W8 add8(const W8& a, const W8& b) {
  W8 r;
  u32 c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = __builtin_addc(a.w[i], b.w[i], c, &c);
  return r;
}

__device__ __forceinline__ W8 sub8(const W8& a, const W8& b, u32* borrow_out = nullptr) {
  W8 r;
  u32 br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = __builtin_subc(a.w[i], b.w[i], br, &br);
  if (borrow_out) *borrow_out = br;
  return r;
}

__device__ __forceinline__ W8 neg8(const W8& a) {
  W8 z;
#pragma unroll
  for (int i = 0; i < 8; i++) z.w[i] = 0;
  return sub8(z, a);
}

// low 256 bits of a*b (schoolbook, 36 partial products).  Each row's products are
// added as two add-with-carry chains (low halves at limb i+j, high halves at i+j+1),
// so no 64-bit addends have to be assembled: 103 VALU instructions instead of 144.
__device__ __forceinline__ W8 mul8(const W8& a, const W8& b) {
  W8 r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u32 lo[8], hi[8];
#pragma unroll
    for (int j = 0; j < 8 - i; j++) {
      const u64 p = (u64)a.w[i] * b.w[j];
      lo[j] = (u32)p;
      hi[j] = (u32)(p >> 32);
    }
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < 8 - i; j++) r.w[i + j] = __builtin_addc(r.w[i + j], lo[j], c, &c);
    c = 0;
#pragma unroll
    for (int j = 0; j + 1 < 8 - i; j++) r.w[i + j + 1] = __builtin_addc(r.w[i + j + 1], hi[j], c, &c);
  }
  return r;
}

// high 256 bits of the 512-bit product.  Row i adds its low halves at limbs i..i+7
// (the chain's carry lands in limb i+8, still zero before this row) and its high
// halves at limbs i+1..i+8; the partial sum after row i fits in i+9 limbs, so the
// high chain's final carry is zero.
__device__ __forceinline__ W8 mulhi8(const W8& a, const W8& b) {
  u32 r[16];
#pragma unroll
  for (int i = 0; i < 16; i++) r[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u32 lo[8], hi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const u64 p = (u64)a.w[i] * b.w[j];
      lo[j] = (u32)p;
      hi[j] = (u32)(p >> 32);
    }
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) r[i + j] = __builtin_addc(r[i + j], lo[j], c, &c);
    r[i + 8] = c;
    c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) r[i + 1 + j] = __builtin_addc(r[i + 1 + j], hi[j], c, &c);
  }
  W8 h;
#pragma unroll
  for (int i = 0; i < 8; i++) h.w[i] = r[i + 8];
  return h;
}

__device__ __forceinline__ bool is_zero8(const W8& a) {
  u32 o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.w[i];
  return o == 0;
}

// a >= b (unsigned)
__device__ __forceinline__ bool uge8(const W8& a, const W8& b) {
  u32 br;
  (void)sub8(a, b, &br);
  return br == 0;
}

__device__ __forceinline__ W8 shl8(const W8& x, u32 s);

// count of leading zero bits of a 256-bit value (256 for zero)
__device__ __forceinline__ u32 clz8(const W8& a) {
  u32 n = 256;
#pragma unroll
  for (int i = 0; i < 8; i++) n = a.w[i] ? (u32)(32 * (7 - i)) + (u32)__builtin_clz(a.w[i]) : n;
  return n;
}

__device__ __forceinline__ W8 shr8(const W8& x, u32 s, u32 fill);

// Restoring division over the quotient bits only.  With la, lb the bit lengths of a and
// b, the quotient has n = la - lb + 1 bits (none if la < lb): the remainder starts as the
// top la - n = lb - 1 bits of a (below b, so the first lb - 1 steps of the textbook loop
// never subtract) and the low n bits of a come in at the top of `quo`, one per step.  The
// remainder keeps NB limbs — every active lane's divisor fits NB limbs and rem < b is the
// loop invariant, so 2*rem+bit needs NB limbs plus the carry bit `c`.  The trip count is
// per lane (the wave runs its longest): a few steps for like-sized operands.
template <int NB>
__device__ __forceinline__ void udivrem_nb(const W8& rem0, const W8& quo0, u32 n, const W8& b, W8& q, W8& r) {
  u32 rem[NB];
#pragma unroll
  for (int i = 0; i < NB; i++) rem[i] = rem0.w[i];
  W8 quo = quo0;
#pragma unroll 1
  for (u32 it = 0; it < n; it++) {
    const u32 c = rem[NB - 1] >> 31;
#pragma unroll
    for (int i = NB - 1; i > 0; i--) rem[i] = __builtin_amdgcn_alignbit(rem[i], rem[i - 1], 31);
    rem[0] = __builtin_amdgcn_alignbit(rem[0], quo.w[7], 31);
#pragma unroll
    for (int i = 7; i > 0; i--) quo.w[i] = __builtin_amdgcn_alignbit(quo.w[i], quo.w[i - 1], 31);
    quo.w[0] <<= 1;
    u32 br = 0, d[NB];
#pragma unroll
    for (int i = 0; i < NB; i++) d[i] = __builtin_subc(rem[i], b.w[i], br, &br);
    const bool ge = (c != 0) | (br == 0);
#pragma unroll
    for (int i = 0; i < NB; i++) rem[i] = ge ? d[i] : rem[i];
    quo.w[0] |= ge ? 1u : 0u;
  }
  q = quo;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = i < NB ? rem[i] : 0u;
}

// q, r of a / b for b != 0 (b == 0: the callers substitute the SMT-LIB results).
// Per lane: a one-limb divisor takes limb-serial long division by reciprocal; a wider one the
// bit-serial loop above, with the remainder width chosen by a ballot over just those lanes.
// The branch is divergent on purpose: in a wave that mixes small and wide divisors each path
// runs for its own lanes only, so a small divisor (hundreds of quotient bits) never drags the
// wide-divisor lanes' loop count up, and vice versa.
__device__ __forceinline__ void udivrem8(const W8& a, const W8& b, W8& q, W8& r) {
  if ((b.w[1] | b.w[2] | b.w[3] | b.w[4] | b.w[5] | b.w[6] | b.w[7]) == 0u) {
    // one-limb divisor: normalised long division, one 2/1 step per limb with the divisor's
    // reciprocal computed once (Moller & Granlund, "Improved division by invariant
    // integers", IEEE TC 2011, Alg. 4): a multiply, a 64-bit add and two corrections per limb
    const u32 d0 = b.w[0] ? b.w[0] : 1u;
    const u32 sh = (u32)__builtin_clz(d0);
    const u32 dn = d0 << sh;  // 2^31 <= dn < 2^32
    const u32 v = (u32)(0xFFFFFFFFFFFFFFFFull / dn - 0x100000000ull);
    u32 rr = sh ? (a.w[7] >> (32u - sh)) : 0u;  // top of the shifted dividend, < 2^sh <= dn
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      const u32 lo = i ? a.w[i - 1] : 0u;
      const u32 ui = sh ? ((a.w[i] << sh) | (lo >> (32u - sh))) : a.w[i];
      const u64 qq = (u64)v * rr + (((u64)rr + 1u) << 32) + ui;  // mod 2^64
      u32 q1 = (u32)(qq >> 32);
      const u32 q0 = (u32)qq;
      u32 r1 = ui - q1 * dn;
      const bool over = r1 > q0;
      q1 = over ? q1 - 1u : q1;
      r1 = over ? r1 + dn : r1;
      const bool ge = r1 >= dn;
      q1 = ge ? q1 + 1u : q1;
      r1 = ge ? r1 - dn : r1;
      q.w[i] = q1;
      rr = r1;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = i ? 0u : (rr >> sh);
  } else {
    const u32 la = 256u - clz8(a), lb = 256u - clz8(b);
    const u32 n = la >= lb ? la - lb + 1u : 0u;  // quotient bits (<= 255 here: lb > 32)
    W8 rem0, quo0;
    if (n == 0) {
#pragma unroll
      for (int i = 0; i < 8; i++) rem0.w[i] = quo0.w[i] = 0;
    } else {
      rem0 = shr8(a, n, 0u);
      quo0 = shl8(a, 256u - n);
    }
    if (__builtin_amdgcn_ballot_w64((b.w[4] | b.w[5] | b.w[6] | b.w[7]) != 0u)) {
      udivrem_nb<8>(rem0, quo0, n, b, q, r);
    } else if (__builtin_amdgcn_ballot_w64((b.w[2] | b.w[3]) != 0u)) {
      udivrem_nb<4>(rem0, quo0, n, b, q, r);
    } else {
      udivrem_nb<2>(rem0, quo0, n, b, q, r);
    }
    if (n == 0) r = a;  // a < b: q = 0, r = a
  }
}

// SMT-LIB bvudiv / bvurem with the total-division convention
__device__ __forceinline__ W8 bv_udiv(const W8& a, const W8& b, u32 width) {
  W8 q, r;
  udivrem8(a, b, q, r);
  if (is_zero8(b)) {
#pragma unroll
    for (int i = 0; i < 8; i++) q.w[i] = 0xFFFFFFFFu;
  }
  canon8(q, width);
  return q;
}

__device__ __forceinline__ W8 bv_urem(const W8& a, const W8& b, u32 width) {
  W8 q, r;
  udivrem8(a, b, q, r);
  if (is_zero8(b)) r = a;
  canon8(r, width);
  return r;
}

__device__ __forceinline__ u32 msb_of(const W8& a, u32 width) {
  const u32 bit = width - 1;
  u32 v = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) v = ((u32)i == (bit >> 5)) ? a.w[i] : v;
  return (v >> (bit & 31)) & 1u;
}

__device__ __forceinline__ W8 negw(const W8& a, u32 width) {
  W8 r = neg8(a);
  canon8(r, width);
  return r;
}

// bvsdiv: msb case split of the SMT-LIB definition
__device__ __forceinline__ W8 bv_sdiv(const W8& a, const W8& b, u32 width) {
  const u32 ma = msb_of(a, width), mb = msb_of(b, width);
  W8 aa = ma ? negw(a, width) : a;
  W8 bb = mb ? negw(b, width) : b;
  W8 q = bv_udiv(aa, bb, width);
  return (ma ^ mb) ? negw(q, width) : q;
}

// bvsrem: sign follows the dividend
__device__ __forceinline__ W8 bv_srem(const W8& a, const W8& b, u32 width) {
  const u32 ma = msb_of(a, width), mb = msb_of(b, width);
  W8 aa = ma ? negw(a, width) : a;
  W8 bb = mb ? negw(b, width) : b;
  W8 r = bv_urem(aa, bb, width);
  return ma ? negw(r, width) : r;
}

// bvsmod: sign follows the divisor
__device__ __forceinline__ W8 bv_smod(const W8& a, const W8& b, u32 width) {
  const u32 ma = msb_of(a, width), mb = msb_of(b, width);
  W8 aa = ma ? negw(a, width) : a;
  W8 bb = mb ? negw(b, width) : b;
  W8 u = bv_urem(aa, bb, width);
  if (is_zero8(u) || (!ma && !mb)) return u;
  W8 r;
  if (ma && !mb) {
    r = add8(negw(u, width), b);
  } else if (!ma && mb) {
    r = add8(u, b);
  } else {
    r = negw(u, width);
  }
  canon8(r, width);
  return r;
}

// shift amount as a saturated small integer: returns width if b >= width
__device__ __forceinline__ u32 shamt(const W8& b, u32 width) {
  u32 hi = 0;
#pragma unroll
  for (int i = 1; i < 8; i++) hi |= b.w[i];
  return (hi != 0 || b.w[0] >= width) ? width : b.w[0];
}

// x << s (s < 256): barrel over whole limbs, then a funnel shift
__device__ __forceinline__ W8 shl8(const W8& x, u32 s) {
  W8 r = x;
  const u32 q = s >> 5, b = s & 31u;
#pragma unroll
  for (int k = 1; k <= 4; k <<= 1) {
    const bool on = (q & (u32)k) != 0;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      u32 v = i - k >= 0 ? r.w[i - k] : 0u;
      r.w[i] = on ? v : r.w[i];
    }
  }
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    u32 lo = i > 0 ? r.w[i - 1] : 0u;
    r.w[i] = (u32)((((u64)r.w[i] << 32) | lo) >> (32 - b));
  }
  return r;
}

// x >> s with fill (0 or ~0) for the vacated bits
__device__ __forceinline__ W8 shr8(const W8& x, u32 s, u32 fill) {
  W8 r = x;
  const u32 q = s >> 5, b = s & 31u;
#pragma unroll
  for (int k = 1; k <= 4; k <<= 1) {
    const bool on = (q & (u32)k) != 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      u32 v = i + k < 8 ? r.w[i + k] : fill;
      r.w[i] = on ? v : r.w[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u32 hi = i < 7 ? r.w[i + 1] : fill;
    r.w[i] = (u32)((((u64)hi << 32) | r.w[i]) >> b);
  }
  return r;
}

__device__ __forceinline__ W8 bv_shl(const W8& a, const W8& b, u32 width) {
  const u32 s = shamt(b, width);
  W8 r;
  if (s >= width) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = 0;
    return r;
  }
  r = shl8(a, s);
  canon8(r, width);
  return r;
}

__device__ __forceinline__ W8 bv_lshr(const W8& a, const W8& b, u32 width) {
  const u32 s = shamt(b, width);
  W8 r;
  if (s >= width) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = 0;
    return r;
  }
  return shr8(a, s, 0u);
}

__device__ __forceinline__ W8 bv_ashr(const W8& a, const W8& b, u32 width) {
  const u32 s = shamt(b, width);
  const u32 neg = msb_of(a, width);
  // sign-extend a to 256 bits, shift with sign fill, re-mask
  W8 x = a;
  if (neg) {
    const u32 L = (width + 31u) >> 5;
    const u32 tm = top_mask(width);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if ((u32)i == L - 1) x.w[i] |= ~tm;
      else if ((u32)i >= L) x.w[i] = 0xFFFFFFFFu;
    }
  }
  W8 r;
  if (s >= width) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = neg ? 0xFFFFFFFFu : 0u;
  } else {
    r = shr8(x, s, neg ? 0xFFFFFFFFu : 0u);
  }
  canon8(r, width);
  return r;
}

// low 256 bits of a*a: 16 doubled cross products + 4 squares (mul8 needs 36),
// accumulated with add-with-carry chains like mul8
__device__ __forceinline__ W8 sqr8(const W8& a) {
  W8 r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    u32 lo[8], hi[8];
#pragma unroll
    for (int j = i + 1; j < 8 - i; j++) {
      const u64 p = (u64)a.w[i] * a.w[j];
      lo[j] = (u32)p;
      hi[j] = (u32)(p >> 32);
    }
    u32 c = 0;
#pragma unroll
    for (int j = i + 1; j < 8 - i; j++) r.w[i + j] = __builtin_addc(r.w[i + j], lo[j], c, &c);
    c = 0;
#pragma unroll
    for (int j = i + 1; j + 1 < 8 - i; j++) r.w[i + j + 1] = __builtin_addc(r.w[i + j + 1], hi[j], c, &c);
  }
#pragma unroll
  for (int i = 7; i > 0; i--) r.w[i] = (r.w[i] << 1) | (r.w[i - 1] >> 31);
  r.w[0] <<= 1;
  W8 d;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const u64 q = (u64)a.w[i] * a.w[i];
    d.w[2 * i] = (u32)q;
    d.w[2 * i + 1] = (u32)(q >> 32);
  }
  return add8(r, d);
}

// EVM EXP (mod 2^width): left-to-right 2-bit fixed-window exponentiation.
// Exponent limbs that are zero in every active lane of the wave are skipped
// (wave-uniform, so no divergence); per 2 exponent bits: two squarings and at
// most one multiply by base^{1,2,3}.
__device__ __forceinline__ W8 bv_exp(const W8& base, const W8& e, u32 width) {
  W8 r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = 0;
  r.w[0] = 1;
  u32 live = 0;  // wave-uniform count of low limbs that are non-zero somewhere
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (__ballot(e.w[i] != 0u) != 0ull) live = i + 1;
  W8 ex = e;
  const u32 sh = 8u - live;  // move the top live limb to limb 7 (uniform barrel stages)
  if (sh & 4u) {
#pragma unroll
    for (int i = 7; i >= 0; i--) ex.w[i] = i >= 4 ? ex.w[i - 4] : 0u;
  }
  if (sh & 2u) {
#pragma unroll
    for (int i = 7; i >= 0; i--) ex.w[i] = i >= 2 ? ex.w[i - 2] : 0u;
  }
  if (sh & 1u) {
#pragma unroll
    for (int i = 7; i >= 0; i--) ex.w[i] = i >= 1 ? ex.w[i - 1] : 0u;
  }
  // the wave's longest exponent inside the top live limb (binary search over ballots), so
  // leading zero digits are skipped too: an 8-bit exponent takes 4 steps, not 16
  u32 m = 0;
  if (live) {
#pragma unroll
    for (u32 step = 16; step >= 1; step >>= 1)
      if (__builtin_amdgcn_ballot_w64((ex.w[7] >> (m + step - 1u)) != 0u)) m += step;
  }
  const u32 skip = (32u - m) & ~1u;  // even: digits stay aligned to the exponent's bit 0
  if (live && skip) ex = shl8(ex, skip);
  const u32 steps = live * 16u - (live ? skip / 2u : 0u);
  const W8 b2 = sqr8(base);
  const W8 b3 = mul8(b2, base);
#pragma unroll 1
  for (u32 it = 0; it < steps; it++) {
    const u32 dg = ex.w[7] >> 30;
#pragma unroll
    for (int i = 7; i > 0; i--) ex.w[i] = (ex.w[i] << 2) | (ex.w[i - 1] >> 30);
    ex.w[0] <<= 2;
    r = sqr8(sqr8(r));
    if (__ballot(dg != 0u) != 0ull) {
      W8 f;
#pragma unroll
      for (int i = 0; i < 8; i++) f.w[i] = dg == 1u ? base.w[i] : (dg == 2u ? b2.w[i] : b3.w[i]);
      const W8 m = mul8(r, f);
#pragma unroll
      for (int i = 0; i < 8; i++) r.w[i] = dg ? m.w[i] : r.w[i];
    }
  }
  canon8(r, width);
  return r;
}

}  // namespace mg

namespace mg {

// low `width` bits of a*b
__device__ __forceinline__ W8 mul8w(const W8& a, const W8& b, u32 width) {
  W8 r = mul8(a, b);
  canon8(r, width);
  return r;
}

// bvumul_noovfl: the full 2w-bit product of two w-bit values fits in w bits
__device__ __forceinline__ u32 umul_noovf8(const W8& x, const W8& y, u32 wa) {
  const W8 lo = mul8(x, y);
  const W8 hi = mulhi8(x, y);
  u32 ov = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    ov |= hi.w[q];
    const u32 bit0 = q * 32;
    u32 m;
    if (bit0 + 32 <= wa) m = 0u;
    else if (bit0 >= wa) m = 0xFFFFFFFFu;
    else m = ~((1u << (wa - bit0)) - 1u);
    ov |= lo.w[q] & m;
  }
  return ov == 0;
}

}  // namespace mg
