// Device helpers for JIT-specialised kernels (compiled at run time by hipRTC
// together with bv_device.h and keccak_device.h; see jit.cpp).
//
// Everything here is indexed with compile-time limb indices (templates on L,
// fully unrolled) so values stay in VGPRs.  The candidate generator primitives
// (gen_device.h) are the same as the interpreter's; jit.cpp inlines the
// per-coordinate generator specialised on its spec.
#pragma once

namespace mg {

// add / subtract with carry for the emitted carry chains.  Default: the hardware carry
// (v_add_co / v_addc_co through VCC).  MG_VGPR_CARRY: the carry as a 0/1 VGPR value —
// s = a + b + c (v_add3_u32), carry-out = bit 31 of (a & b) | ((a | b) & ~s) (one v_bitop3_b32,
// table 0xD4) — which has no VALU-writes-SGPR -> VALU-reads hazard between links.
__device__ __forceinline__ uint32_t mg_addc(uint32_t a, uint32_t b, uint32_t ci, uint32_t* co) {
#ifdef MG_VGPR_CARRY
  const uint32_t s = a + b + ci;
  *co = __builtin_amdgcn_bitop3_b32(a, b, s, 0xD4) >> 31;
  return s;
#else
  return __builtin_addc(a, b, ci, co);
#endif
}

// borrow-out = bit 31 of (~a & b) | (~(a ^ b) & d) (table 0x8E)
__device__ __forceinline__ uint32_t mg_subc(uint32_t a, uint32_t b, uint32_t bi, uint32_t* bo) {
#ifdef MG_VGPR_CARRY
  const uint32_t d = a - b - bi;
  *bo = __builtin_amdgcn_bitop3_b32(a, b, d, 0x8E) >> 31;
  return d;
#else
  return __builtin_subc(a, b, bi, bo);
#endif
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
