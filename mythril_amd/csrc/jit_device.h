// Device helpers for JIT-specialised kernels (compiled at run time by hipRTC
// together with bv_device.h and keccak_device.h; see jit.cpp).
//
// Everything here is indexed with compile-time limb indices (templates on L,
// fully unrolled) so values stay in VGPRs.  The candidate generator is the
// same pure function of (seed, index, coordinate) as the interpreter's
// (engine.hip gen_coord) — tests check the two paths candidate by candidate.
#pragma once

namespace mg {

struct GenSpec {
  uint32_t kind, p[7];
};

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t cand_key(uint64_t idx, uint64_t seed) {
  return mix32((uint32_t)idx ^
               mix32((uint32_t)(idx >> 32) ^ (uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + 0x632BE5ABu)));
}

__device__ __forceinline__ uint32_t rnd(uint32_t key, uint32_t c, uint32_t j) {
  /* one-multiply finaliser of the (well mixed) candidate key; see MG_GEN_* in mythgpu.h */
  uint32_t x = key ^ (c * 0x9E3779B9u + j * 0x85EBCA6Bu + 0x27D4EB2Fu);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  return x;
}

// MG_GEN_* kinds (include/mythgpu.h)
enum : uint32_t { G_UNIFORM = 0, G_RANGE = 1, G_DICT = 2, G_MIXED = 3, G_ALIGNED = 4, G_FIXED = 5, G_LAZY = 6 };

template <int L>
__device__ __forceinline__ void gen_regs(uint32_t (&o)[L], const uint32_t* __restrict__ gconsts,
                                         const GenSpec* __restrict__ specs, const uint32_t* __restrict__ cw,
                                         uint32_t c, uint32_t width, uint32_t key) {
  uint32_t cc = c;
  GenSpec s = specs[c];
  const uint32_t fix_dst = s.kind >> 8;
  uint32_t fix_src = 0;
  s.kind &= 0xFFu;
  uint32_t Lg = L;
  bool allow_copy = true;
  bool from_mixed = false;
#pragma unroll
  for (int level = 0; level < 2; level++) {
    if (s.kind != G_MIXED) break;
    const uint32_t h = rnd(key, cc, 0xFFFFu);
    const uint32_t sel = h & 0xFFFFu;
    const bool narrow = cw[cc] <= 16u;  // MG_GEN_NARROW_BITS: uniform / small value from h >> 16
    const uint32_t pc = (allow_copy && s.p[3] != 0xFFFFFFFFu) ? s.p[4] : 0u;
    const uint32_t pd = s.p[1] ? s.p[2] : 0u;
    const uint32_t ps = s.p[6] & 0xFFFFu;
    if (sel < pc) {
      cc = s.p[3];
      s = specs[cc];
      fix_src = s.kind >> 8;
      s.kind &= 0xFFu;
      const uint32_t Ls = (cw[cc] + 31) >> 5;
      Lg = Ls < (uint32_t)L ? Ls : (uint32_t)L;
      allow_copy = false;
      continue;
    }
    if (sel < pc + pd) {
      s.kind = G_DICT;
      from_mixed = true;
    } else if (sel < pc + pd + ps) {
      const uint32_t bits = (s.p[6] >> 16) < width ? (s.p[6] >> 16) : width;
#pragma unroll
      for (int j = 0; j < L; j++) {
        uint32_t v = narrow ? (j == 0 ? h >> 16 : 0u) : rnd(key, cc, j);
        const uint32_t lo = j * 32;
        o[j] = lo >= bits ? 0u : (bits - lo >= 32 ? v : (v & ((1u << (bits - lo)) - 1u)));
      }
      s.kind = 0xFFu;  // done
    } else if (narrow) {
#pragma unroll
      for (int j = 0; j < L; j++) o[j] = j == 0 ? h >> 16 : 0u;
      s.kind = 0xFFu;  // done
    } else {
      s.kind = G_UNIFORM;
    }
    break;
  }
  const uint32_t Ls = (cw[cc] + 31) >> 5;
  switch (s.kind) {
    case 0xFFu:
      break;
    case G_DICT: {
      const uint32_t e = (((rnd(key, cc, 0xFFFFu) >> 16) * s.p[1]) >> 16);
      const uint32_t* src = gconsts + s.p[0] + e * Ls;
#pragma unroll
      for (int j = 0; j < L; j++) o[j] = (uint32_t)j < Lg ? src[j] : 0u;
      if (from_mixed && s.p[5]) {
        const uint32_t r = rnd(key, cc, 0u);
        if ((r & 0xFFFFu) < s.p[5]) {
          const uint32_t mag = ((r >> 16) & 1u) + 1u;
          const bool sub = (r >> 17) & 1u;
          uint64_t carry = mag;
#pragma unroll
          for (int j = 0; j < L; j++) {
            if ((uint32_t)j < Lg) {
              const uint64_t t = sub ? ((uint64_t)o[j] - carry) : ((uint64_t)o[j] + carry);
              o[j] = (uint32_t)t;
              carry = sub ? ((t >> 32) & 1u) : (t >> 32);
            }
          }
        }
      }
      break;
    }
    case G_RANGE: {
      const uint32_t span = s.p[1];
      const uint32_t r = rnd(key, cc, 0);
      const uint32_t off = span ? (uint32_t)(((uint64_t)r * span) >> 32) : r;
      uint64_t carry = off;
#pragma unroll
      for (int j = 0; j < L; j++) {
        if ((uint32_t)j < Lg) {
          const uint64_t t = (uint64_t)gconsts[s.p[0] + j] + carry;
          o[j] = (uint32_t)t;
          carry = t >> 32;
        } else {
          o[j] = 0;
        }
      }
      break;
    }
    case G_ALIGNED: {
      const uint32_t cnt = s.p[2];
      const uint32_t r = rnd(key, cc, 0);
      const uint64_t m = cnt ? (((uint64_t)r * cnt) >> 32) : r;
      const uint32_t sh = s.p[1];
      uint64_t carry = 0;
#pragma unroll
      for (int j = 0; j < L; j++) {
        if ((uint32_t)j < Lg) {
          const int32_t bit0 = (int32_t)(j * 32) - (int32_t)sh;
          uint32_t mw;
          if (bit0 <= -32 || bit0 >= 64) mw = 0;
          else if (bit0 < 0) mw = (uint32_t)(m << (-bit0));
          else mw = (uint32_t)(m >> bit0);
          const uint64_t t = (uint64_t)gconsts[s.p[0] + j] + mw + carry;
          o[j] = (uint32_t)t;
          carry = t >> 32;
        } else {
          o[j] = 0;
        }
      }
      break;
    }
    case G_FIXED: {
#pragma unroll
      for (int j = 0; j < L; j++) o[j] = (uint32_t)j < Lg ? gconsts[s.p[0] + j] : 0u;
      break;
    }
    default: {
#pragma unroll
      for (int j = 0; j < L; j++) o[j] = (uint32_t)j < Lg ? rnd(key, cc, j) : 0u;
      break;
    }
  }
  // a copy is the source's value: masked to the source width, then truncated / zero-extended
  if (cc != c && Lg == Ls && (cw[cc] & 31u)) {
#pragma unroll
    for (int j = 0; j < L; j++)
      if ((uint32_t)j == Lg - 1) o[j] &= (1u << (cw[cc] & 31u)) - 1u;
  }
  const uint32_t r = width & 31u;
  if (r) o[L - 1] &= (1u << r) - 1u;
  if (cc != c && fix_src) {
    const uint32_t* f = gconsts + (fix_src - 1);
#pragma unroll
    for (int j = 0; j < L; j++)
      if ((uint32_t)j < Lg) o[j] = (o[j] & ~f[j]) | f[Ls + j];
  }
  if (fix_dst) {
    const uint32_t* f = gconsts + (fix_dst - 1);
#pragma unroll
    for (int j = 0; j < L; j++) o[j] = (o[j] & ~f[j]) | f[L + j];
  }
}

// Keccak-256 of the LEN big-endian bytes of an L-limb value (LEN >= 1)
template <int L, int LEN>
__device__ __forceinline__ void keccak_value(const uint32_t (&in)[L], uint32_t (&out)[8]) {
  uint64_t st[25];
#pragma unroll
  for (int i = 0; i < 25; i++) st[i] = 0;
  constexpr int NB = LEN / 136 + 1;
#pragma unroll
  for (int b = 0; b < NB; b++) {
#pragma unroll
    for (int t = 0; t < 17; t++) {
      uint64_t lane = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int m = b * 136 + t * 8 + k;
        uint32_t byte = 0;
        if (m < LEN) {
          const int bitpos = 8 * (LEN - 1 - m);
          byte = (in[bitpos >> 5] >> (bitpos & 31)) & 0xFFu;
        }
        if (m == LEN) byte |= 0x01u;
        if (m == NB * 136 - 1) byte |= 0x80u;
        lane |= (uint64_t)byte << (8 * k);
      }
      st[t] ^= lane;
    }
    keccak_f1600(st);
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int q = 7 - j;
    const uint32_t d = (q & 1) ? (uint32_t)(st[q >> 1] >> 32) : (uint32_t)st[q >> 1];
    out[j] = __builtin_bswap32(d);
  }
}

}  // namespace mg
