// Device helpers for JIT-specialised kernels (compiled at run time by hipRTC
// together with bv_device.h and keccak_device.h; see jit.cpp).
//
// Everything here is indexed with compile-time limb indices (templates on L,
// fully unrolled) so values stay in VGPRs.  The candidate generator primitives
// (gen_device.h) are the same as the interpreter's; jit.cpp inlines the
// per-coordinate generator specialised on its spec.
#pragma once

namespace mg {

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
