// GEN3 candidate-generator primitives (format in include/mythgpu.h), shared by the
// interpreter kernels (engine.hip), the JIT prelude (jit.cpp -> hipRTC) and the host
// (seed keys are folded once per launch on the CPU and passed as kernel arguments).
//
// Two keys per candidate index i:
//   G = fmix64((i >> 6) ^ SG)      per aligned group of 64 indices = one wave: the MIXED
//                                  alternative, so the choice is a scalar (SGPR) branch
//   K = G ^ fmix64((i & 63) ^ SK)  per lane: limb / index / delta bits.  The lane half
//                                  depends on the lane only, so a kernel computes it once
//                                  and pays one 64-bit XOR per group (GEN2 hashed i itself)
#pragma once

namespace mg {

__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return x;
}

__host__ __device__ __forceinline__ uint64_t seed_lane_key(uint64_t seed) { return fmix64(seed ^ 0x6A09E667F3BCC908ull); }
__host__ __device__ __forceinline__ uint64_t seed_group_key(uint64_t seed) { return fmix64(seed ^ 0xBB67AE8584CAA73Bull); }

__host__ __device__ __forceinline__ uint32_t gsalt(uint32_t c, uint32_t j) {
  return c * 0x9E3779B9u + j * 0x85EBCA6Bu + 0x27D4EB2Fu;
}

// xorshift-multiply-xorshift; the multiply takes 24 bits (v_mul_u32_u24, a full-rate VALU
// op; the 32-bit v_mul_lo_u32 issues at a quarter of the rate).  Every input bit still
// reaches the product: bits 24..31 come in through x ^ (x >> 16).
__host__ __device__ __forceinline__ uint32_t gfin(uint32_t x) {
  x ^= x >> 16;
  x = (x & 0xFFFFFFu) * 0x9E3779u;
  x ^= x >> 15;
  return x;
}

// raw limb j >= 2 of a UNIFORM value from its raw limbs j-1 (a) and j-2 (b): a funnel
// shift of a:b (v_alignbit_b32) plus b — two VALU instructions where a hashed limb takes
// five; limbs 0 and 1 are hashed (grnd)
__host__ __device__ __forceinline__ uint32_t gext(uint32_t a, uint32_t b, uint32_t j) {
  const uint32_t s = (7u * j + 3u) % 31u + 1u;  // 1..31
  return (uint32_t)(((((uint64_t)a) << 32) | b) >> s) + b;
}

// kf = klo ^ (klo >> 16): gfin's first xor-shift is linear, so (klo ^ salt) ^ ((klo ^ salt) >> 16) =
// kf ^ (salt ^ (salt >> 16)) — the key's half folded once per group, each draw XORs in its salt's
// fold (a constant in the compiled kernels, a scalar in the interpreter): one vector op per draw
struct GKeys {
  uint32_t klo, khi, glo, ghi, kf;
};

// lk = gen_lane_key(idx & 63, sk), computed once per lane by kernels whose lanes keep their slot
__device__ __forceinline__ uint64_t gen_lane_key(uint64_t lane, uint64_t sk) { return fmix64(lane ^ sk); }

__device__ __forceinline__ GKeys gen_keys_lk(uint64_t idx, uint64_t lk, uint64_t sg) {
  const uint64_t G = fmix64((idx >> 6) ^ sg);
  const uint64_t K = G ^ lk;
  GKeys k;
  k.klo = (uint32_t)K;
  k.khi = (uint32_t)(K >> 32);
  k.kf = k.klo ^ (k.klo >> 16);
  k.glo = (uint32_t)G;
  k.ghi = (uint32_t)(G >> 32);
  return k;
}

__device__ __forceinline__ GKeys gen_keys(uint64_t idx, uint64_t sk, uint64_t sg) {
  return gen_keys_lk(idx, gen_lane_key(idx & 63u, sk), sg);
}

// per-lane random limb j of coordinate c; h(c) = grnd(k, c, 0xFFFF)
__device__ __forceinline__ uint32_t grnd(const GKeys& k, uint32_t c, uint32_t j) {
  const uint32_t s = gsalt(c, j);
  uint32_t x = k.kf ^ (s ^ (s >> 16));  // = (klo ^ s) ^ ((klo ^ s) >> 16), gfin's first step
  x = (x & 0xFFFFFFu) * 0x9E3779u;
  x ^= x >> 15;
  return x + k.khi;
}

// per-group choice bits of coordinate c (high 16: alternative, low 16: delta).  Wave-uniform,
// so it runs on the scalar unit, which every SIMD of the CU shares: a multiply-add (3 SALU)
// instead of the lane finaliser (9 SALU), and the alternative comes from the better-mixed
// high half of the product
__device__ __forceinline__ uint32_t gwsel(const GKeys& k, uint32_t c) {
  return (k.glo ^ gsalt(c, 0xFFFEu)) * 0x9E3779B1u + k.ghi;
}

}  // namespace mg
