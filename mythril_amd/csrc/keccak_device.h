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

__device__ __forceinline__ uint64_t rol64(uint64_t v, int n) { return (v << n) | (v >> (64 - n)); }

__device__ __forceinline__ void keccak_f1600(uint64_t (&a)[25]) {
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    uint64_t c0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20];
    uint64_t c1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];
    uint64_t c2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22];
    uint64_t c3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];
    uint64_t c4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];
    uint64_t d0 = c4 ^ rol64(c1, 1), d1 = c0 ^ rol64(c2, 1), d2 = c1 ^ rol64(c3, 1), d3 = c2 ^ rol64(c4, 1),
             d4 = c3 ^ rol64(c0, 1);
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      a[y + 0] ^= d0; a[y + 1] ^= d1; a[y + 2] ^= d2; a[y + 3] ^= d3; a[y + 4] ^= d4;
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
      uint64_t b0 = a[y], b1 = a[y + 1], b2 = a[y + 2], b3 = a[y + 3], b4 = a[y + 4];
      a[y + 0] = b0 ^ (~b1 & b2);
      a[y + 1] = b1 ^ (~b2 & b3);
      a[y + 2] = b2 ^ (~b3 & b4);
      a[y + 3] = b3 ^ (~b4 & b0);
      a[y + 4] = b4 ^ (~b0 & b1);
    }
    a[0] ^= kKeccakRC[round];
  }
}

}  // namespace mg
