// Keccak-f[1600] for one lane (state in 50 VGPRs as 25 x u64).
// Rotation offsets / round constants are the published Keccak parameters
// (the reference obtains the hash from ethereum.utils.sha3,
// mythril/laser/ethereum/keccak_function_manager.py:44-57).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mg {

__device__ __constant__ static const uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

// 64-bit lanes as (lo, hi) 32-bit halves.  gfx950 has no 64-bit rotate; a
// rotate is two v_alignbit_b32 (funnel shifts), 3-input XOR / chi's
// a ^ (~b & c) are single v_bitop3_b32 (truth tables 0x96 / 0xD2).
__device__ __forceinline__ uint32_t lo32(uint64_t v) { return (uint32_t)v; }
__device__ __forceinline__ uint32_t hi32(uint64_t v) { return (uint32_t)(v >> 32); }
__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

__device__ __forceinline__ uint64_t rol64(uint64_t v, int n) {
  const uint32_t l = lo32(v), h = hi32(v);
  if (n == 32) return mk64(h, l);
  if (n < 32)
    return mk64(__builtin_amdgcn_alignbit(l, h, 32 - n), __builtin_amdgcn_alignbit(h, l, 32 - n));
  return mk64(__builtin_amdgcn_alignbit(h, l, 64 - n), __builtin_amdgcn_alignbit(l, h, 64 - n));
}

__device__ __forceinline__ uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  return mk64(xor3_32(lo32(a), lo32(b), lo32(c)), xor3_32(hi32(a), hi32(b), hi32(c)));
}

__device__ __forceinline__ uint64_t xor5(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e) {
  return mk64(xor3_32(xor3_32(lo32(a), lo32(b), lo32(c)), lo32(d), lo32(e)),
              xor3_32(xor3_32(hi32(a), hi32(b), hi32(c)), hi32(d), hi32(e)));
}

// a ^ (~b & c)
__device__ __forceinline__ uint64_t chi64(uint64_t a, uint64_t b, uint64_t c) {
  return mk64(__builtin_amdgcn_bitop3_b32(lo32(a), lo32(b), lo32(c), 0xD2),
              __builtin_amdgcn_bitop3_b32(hi32(a), hi32(b), hi32(c), 0xD2));
}

__device__ __forceinline__ void keccak_f1600(uint64_t (&a)[25]) {
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    const uint64_t c0 = xor5(a[0], a[5], a[10], a[15], a[20]);
    const uint64_t c1 = xor5(a[1], a[6], a[11], a[16], a[21]);
    const uint64_t c2 = xor5(a[2], a[7], a[12], a[17], a[22]);
    const uint64_t c3 = xor5(a[3], a[8], a[13], a[18], a[23]);
    const uint64_t c4 = xor5(a[4], a[9], a[14], a[19], a[24]);
    // a[x] ^= C[x-1] ^ rot(C[x+1], 1): one 3-input XOR per half instead of forming D first
    const uint64_t r0 = rol64(c0, 1), r1 = rol64(c1, 1), r2 = rol64(c2, 1), r3 = rol64(c3, 1), r4 = rol64(c4, 1);
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      a[y + 0] = xor3_64(a[y + 0], c4, r1);
      a[y + 1] = xor3_64(a[y + 1], c0, r2);
      a[y + 2] = xor3_64(a[y + 2], c1, r3);
      a[y + 3] = xor3_64(a[y + 3], c2, r4);
      a[y + 4] = xor3_64(a[y + 4], c3, r0);
    }
    // rho + pi: b[y, 2x+3y] = rot(a[x, y], r[x, y]) — unrolled along the pi cycle
    uint64_t t = a[1], u;
    u = a[10]; a[10] = rol64(t, 1);  t = u;
    u = a[7];  a[7]  = rol64(t, 3);  t = u;
    u = a[11]; a[11] = rol64(t, 6);  t = u;
    u = a[17]; a[17] = rol64(t, 10); t = u;
    u = a[18]; a[18] = rol64(t, 15); t = u;
    u = a[3];  a[3]  = rol64(t, 21); t = u;
    u = a[5];  a[5]  = rol64(t, 28); t = u;
    u = a[16]; a[16] = rol64(t, 36); t = u;
    u = a[8];  a[8]  = rol64(t, 45); t = u;
    u = a[21]; a[21] = rol64(t, 55); t = u;
    u = a[24]; a[24] = rol64(t, 2);  t = u;
    u = a[4];  a[4]  = rol64(t, 14); t = u;
    u = a[15]; a[15] = rol64(t, 27); t = u;
    u = a[23]; a[23] = rol64(t, 41); t = u;
    u = a[19]; a[19] = rol64(t, 56); t = u;
    u = a[13]; a[13] = rol64(t, 8);  t = u;
    u = a[12]; a[12] = rol64(t, 25); t = u;
    u = a[2];  a[2]  = rol64(t, 43); t = u;
    u = a[20]; a[20] = rol64(t, 62); t = u;
    u = a[14]; a[14] = rol64(t, 18); t = u;
    u = a[22]; a[22] = rol64(t, 39); t = u;
    u = a[9];  a[9]  = rol64(t, 61); t = u;
    u = a[6];  a[6]  = rol64(t, 20); t = u;
    a[1] = rol64(t, 44);
    // chi
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      const uint64_t b0 = a[y], b1 = a[y + 1], b2 = a[y + 2], b3 = a[y + 3], b4 = a[y + 4];
      a[y + 0] = chi64(b0, b1, b2);
      a[y + 1] = chi64(b1, b2, b3);
      a[y + 2] = chi64(b2, b3, b4);
      a[y + 3] = chi64(b3, b4, b0);
      a[y + 4] = chi64(b4, b0, b1);
    }
    a[0] ^= kKeccakRC[round];
  }
}

}  // namespace mg
