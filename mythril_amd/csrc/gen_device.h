// GEN2 candidate-generator primitives (format in include/mythgpu.h), shared by the
// interpreter kernels (engine.hip), the JIT prelude (jit.cpp -> hipRTC) and the host
// (seed keys are folded once per launch on the CPU and passed as kernel arguments).
//
// Two keys per candidate index i:
//   K = fmix64(i ^ SK)        per lane: limb / index / delta bits
//   G = fmix64((i >> 6) ^ SG) per aligned group of 64 indices = one wave: the MIXED
//                             alternative, so the choice is a scalar (SGPR) branch
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

__host__ __device__ __forceinline__ uint32_t gfin(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  return x;
}

struct GKeys {
  uint32_t klo, khi, glo, ghi;
};

__device__ __forceinline__ GKeys gen_keys(uint64_t idx, uint64_t sk, uint64_t sg) {
  const uint64_t K = fmix64(idx ^ sk);
  const uint64_t G = fmix64((idx >> 6) ^ sg);
  GKeys k;
  k.klo = (uint32_t)K;
  k.khi = (uint32_t)(K >> 32);
  k.glo = (uint32_t)G;
  k.ghi = (uint32_t)(G >> 32);
  return k;
}

// per-lane random limb j of coordinate c; h(c) = grnd(k, c, 0xFFFF)
__device__ __forceinline__ uint32_t grnd(const GKeys& k, uint32_t c, uint32_t j) {
  return gfin(k.klo ^ gsalt(c, j)) + k.khi;
}

// per-group choice bits of coordinate c (low 16: alternative, high 16: delta)
__device__ __forceinline__ uint32_t gwsel(const GKeys& k, uint32_t c) { return gfin(k.glo ^ gsalt(c, 0xFFFEu)) + k.ghi; }

}  // namespace mg
