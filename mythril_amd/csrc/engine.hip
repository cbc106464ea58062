// MI355X batched bit-vector evaluation engine: kernels + C-ABI (libmythgpu.so).
//
// One lane evaluates one candidate assignment.  The lowered program
// (program.cpp) is wave-uniform: each 32-byte instruction is fetched with scalar
// loads and dispatched with scalar branches; values live in a per-lane value
// file laid out [word][lane] (LDS when it fits, else an HBM/L2 scratch slab), so
// every value-file access is a conflict-free / fully coalesced 4-byte-per-lane
// access.  256-bit arithmetic (MUL/DIV/shift/EXP) is done in VGPRs
// (bv_device.h); linear ops (ADD/SUB/logic/compare/concat/extract) stream words.
//
// Modes: EVAL (coordinates from a SoA buffer in HBM), GEN (coordinates from the
// counter-based generator, for model materialisation), SEARCH (generator + wave
// ballot + atomicMin first hit).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <list>
#include <thread>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mythgpu.h"
#include "bv_device.h"
#include "keccak_device.h"
#include "gen_device.h"
#include "jit.hpp"
#include "program.hpp"

namespace mg {

constexpr int kWave = 64;
constexpr size_t kCaptureBytes = 64ull << 20;  // watch-row capture buffer (mg_search), per device
// value file in LDS up to this many words per lane (160: 40 KiB per wave), else in global memory;
// MYTHGPU_INTERP_LDS_MAX overrides (at most 255: 64 KiB per one-wave block)
// The hit buffer: [0] the first hit, [1] a hit count, then kHitStripes more counts, one per
// 128-byte line (u64 index kHitStride * (1 + s)).  A search kernel adds a wave's (or block's) hits
// to the stripe of its block: every wave of a launch finishes in its last few percent and their
// adds on one address serialised there; the host sums the stripes.
constexpr uint32_t kHitStripes = 16, kHitStride = 16;
constexpr uint32_t kHitWords = kHitStride * (1 + kHitStripes);
// After them (never armed, never read back) the device's peer line: [0] n, [1 + k] the hit word of
// the k-th device whose slice lies above this one's (in-process multi-device searches).  A wave
// that publishes an early-exit first hit also lowers those words, so their waves, all above the
// hit, stop at their next group boundary instead of sweeping to the end of their slice (the host
// min over the devices is unchanged: the lowest hit is in this device's own word).  Written by
// mg_init; jit.cpp and jit_asm.cpp read it at the same offset (kPeerWord, 2,176 B).
constexpr uint32_t kPeerWord = kHitWords, kPeerMax = 15;
constexpr uint32_t kHitAlloc = kHitWords + 1 + kPeerMax;
// mg_jit_search_many: launches per batch (one hit buffer each) and the streams they alternate on
constexpr uint32_t kManySlots = 64;
constexpr int kManyStreams = 4;
static_assert(kPeerWord == 272, "jit.cpp / jit_asm.cpp hard-code the peer line at 2,176 B");

// mg_init's warm-up thread (helper processes started, one tiny kernel assembled): detached, counted
// here, and waited for by mg_shutdown and the exit handler before they stop the helpers, so a
// shutdown never races the warm-up's helper I/O
static std::mutex g_warm_mu;
static std::condition_variable g_warm_cv;
static int g_warm_running = 0;
static void wait_warm() {
  std::unique_lock<std::mutex> wl(g_warm_mu);
  g_warm_cv.wait_for(wl, std::chrono::seconds(30), [] { return g_warm_running == 0; });
}

// an early-exit first hit to the devices above this one (the peer line).  System scope (gfx950:
// global_atomic_umin_x2 ... sc1): a peer's word may live on another GPU, in fine-grained memory
// (mg_init allocates every hit buffer fine-grained when the mask spans physical devices), where the
// atomic is performed at the owner's memory and its waves' system-scope loads see it
__device__ __forceinline__ void publish_peers(unsigned long long* hit, unsigned long long v) {
  const unsigned long long* t = hit + kPeerWord;
  const uint32_t np = (uint32_t)t[0];
  for (uint32_t q = 0; q < np && q < kPeerMax; q++)
    __hip_atomic_fetch_min((unsigned long long*)t[1 + q], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// the launch's current first hit: agent scope, or system scope when peers on other GPUs lower it
__device__ __forceinline__ unsigned long long read_first_hit(const unsigned long long* hit, uint32_t flags) {
  if (flags & MG_SEARCH_SYSTEM_SCOPE) return __hip_atomic_load(hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return __hip_atomic_load(hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static uint32_t lds_words_max() {
  static const uint32_t n = [] {
    const char* g = getenv("MYTHGPU_INTERP_LDS_MAX");
    const int v = g ? atoi(g) : 160;
    return (uint32_t)std::max(1, std::min(v, 255));
  }();
  return n;
}

__device__ __constant__ static const uint32_t kEmptyKeccak[8] = {
    0x5d85a470u, 0x7bfad804u, 0xca82273bu, 0xe500b653u, 0xdcc703c0u, 0x927e7db2u, 0x86f7233cu, 0xc5d24601u};

enum Mode : int { MODE_EVAL = 0, MODE_GEN = 1, MODE_SEARCH = 2 };

// Program data (instructions, literals, generator specs) is read-only for a kernel's
// lifetime.  Reading it through the constant address space lets the compiler use
// scalar loads (and the scalar cache) for every wave-uniform read; through a generic
// pointer it must assume the kernel's own stores may alias and fetches every
// interpreted instruction with a vector load (measured: ~2,000 cycles per op).
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* cst(const T* p) {
  return (const __attribute__((address_space(4))) T*)p;
}

struct KArgs {
  const Instr* code;
  const uint32_t* consts;
  const uint32_t* aux;
  const GenSpec* specs;
  const uint32_t* gconsts;
  const uint32_t* coord_width;
  const uint32_t* soa;       // EVAL: [row][n]
  uint8_t* verdict;          // EVAL/GEN: [n]
  uint32_t* watch;           // EVAL/GEN: [row][n] (nullable)
  uint32_t* scratch;         // global value file [word][stride]
  unsigned long long* first_hit;
  unsigned long long* hits;
  uint64_t start, count, seed, stride;
  uint64_t sk, sg;           // GEN3 seed keys (seed_lane_key / seed_group_key of seed)
  uint32_t n_instr, value_words, flags;
  uint32_t watch_words;      // SEARCH with `watch`: rows per block of the capture buffer (see K_WATCH)
  uint32_t n_specs;          // generator specs (coordinates): the prologue's scalar-cache warm-up
  uint32_t pc0;              // code[0, pc0): hoisted K_CONSTs, run once per thread (Lowered::n_hoisted)
  uint32_t n_gconsts;        // words at gconsts
  uint32_t lds_g;            // word offset of the prologue's LDS copy of gconsts (kNoLds: none)
};
constexpr uint32_t kNoLds = 0xFFFFFFFFu;

// the dynamic LDS of k_run: the value file (VFLds), then the generator constants' copy (lds_g)
extern __shared__ uint32_t mg_lds[];

// word i of the generator constants at a per-lane index: from the block's LDS copy when the
// prologue staged one (a gather from global memory is an L2 round trip per dictionary limb)
__device__ __forceinline__ uint32_t gword(const KArgs& k, uint32_t i) {
  return k.lds_g != kNoLds ? mg_lds[k.lds_g + i] : cst(k.gconsts)[i];
}

constexpr uint32_t kFlagPrefetch = 1u << 16;
constexpr int kTierLight = 0, kTierMid = 1, kTierHeavy = 2;  // KArgs::flags: warm the scalar cache first (launch_async)

// uniform struct reads through the constant address space (scalar loads)
__device__ __forceinline__ GenSpec ld_spec(const KArgs& k, uint32_t c) {
  const auto* p = cst((const uint32_t*)k.specs) + 8u * c;
  GenSpec s;
  s.kind = p[0];
#pragma unroll
  for (int q = 0; q < 7; q++) s.p[q] = p[1 + q];
  return s;
}

__device__ __forceinline__ Instr ld_instr(const KArgs& k, uint32_t pc) {
  const auto* p = cst((const uint32_t*)k.code) + 8u * pc;
  // wave-uniform by construction: keep every field in SGPRs (a scalar opcode switch)
  Instr in;
  uint32_t* f = &in.op;
#pragma unroll
  for (int q = 0; q < 8; q++) f[q] = (uint32_t)__builtin_amdgcn_readfirstlane((int)p[q]);
  return in;
}


// ---------------------------------------------------------------------------
// value file policies
// ---------------------------------------------------------------------------
struct VFLds {
  uint32_t* base;
  __device__ VFLds(uint32_t* lds, const KArgs&) : base(lds) {}
  __device__ __forceinline__ uint32_t& at(uint32_t w) const { return base[w * kWave + threadIdx.x]; }
};

struct VFGlobal {
  uint32_t* base;
  uint64_t stride;
  __device__ VFGlobal(uint32_t*, const KArgs& k)
      : base(k.scratch + (uint64_t)blockIdx.x * kWave + threadIdx.x), stride(k.stride) {}
  __device__ __forceinline__ uint32_t& at(uint32_t w) const { return base[(uint64_t)w * stride]; }
};

// 256-bit values with every source limb loaded before any result limb is stored.  LDS runs a wave's
// operations in order, but the compiler cannot move the load of a + j + 1 above the store to dst + j
// (they may alias), so a limb-interleaved handler paid one LDS round trip per limb
template <class VF>
__device__ __forceinline__ void lda8(const VF& vf, uint32_t off, uint32_t* x) {
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = vf.at(off + j);
}
template <class VF>
__device__ __forceinline__ void sta8(const VF& vf, uint32_t off, const uint32_t* x) {
#pragma unroll
  for (int j = 0; j < 8; j++) vf.at(off + j) = x[j];
}

// ---------------------------------------------------------------------------
// candidate generator, GEN3 (include/mythgpu.h): a pure function of (seed, index,
// coordinate); the same function as oracle/bveval.c gen_value and the JIT's
// straight-line gen_value (jit.cpp), checked candidate by candidate by the tests
// ---------------------------------------------------------------------------
enum : uint32_t { ALT_NONE = 0, ALT_COPY = 1, ALT_DICT = 2, ALT_SMALL = 3, ALT_UNIFORM = 4 };

__device__ __forceinline__ uint32_t mixed_alt(const GenSpec& s, uint32_t ws) {
  const uint32_t sel = ws >> 16;
  const uint32_t pc = s.p[3] != MG_NONE ? (s.p[2] & 0xFFFFu) : 0u;
  const uint32_t pd = s.p[1] ? (s.p[2] >> 16) : 0u;
  const uint32_t ps = s.p[4] & 0xFFFFu;
  return sel < pc ? ALT_COPY : sel < pc + pd ? ALT_DICT : sel < pc + pd + ps ? ALT_SMALL : ALT_UNIFORM;
}

// value of coordinate c before its finish (MIXED: the chosen non-COPY alternative)
template <class VF>
__device__ __forceinline__ void gen_base(const KArgs& k, const VF& vf, uint32_t dst, uint32_t c, uint32_t width, const GKeys& ky,
                         const GenSpec& s, uint32_t alt) {
  const uint32_t L = (width + 31) >> 5;
  switch (MG_GEN_KIND(s.kind)) {
    case MG_GEN_RANGE: {
      const uint32_t span = s.p[1], r = grnd(ky, c, 0);
      uint32_t off = span ? (uint32_t)(((uint64_t)r * span) >> 32) : r, cy = 0;
      for (uint32_t j = 0; j < L; j++) {
        vf.at(dst + j) = __builtin_addc(cst(k.gconsts)[s.p[0] + j], j ? 0u : off, cy, &cy);
      }
      break;
    }
    case MG_GEN_DICT: {
      const uint32_t e = ((grnd(ky, c, 0xFFFFu) >> 16) * s.p[1]) >> 16;
      if (L == 8) {  // the entry's limbs first, then the stores (gword may read LDS: no interleaving)
        uint32_t x[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) x[j] = gword(k, s.p[0] + e * 8 + j);
        sta8(vf, dst, x);
      } else {
        for (uint32_t j = 0; j < L; j++) vf.at(dst + j) = gword(k, s.p[0] + e * L + j);
      }
      break;
    }
    case MG_GEN_ALIGNED: {
      const uint32_t cnt = s.p[2], r = grnd(ky, c, 0);
      const uint64_t m = cnt ? (((uint64_t)r * cnt) >> 32) : r;
      const uint32_t sh = s.p[1];
      uint32_t cy = 0;
      for (uint32_t j = 0; j < L; j++) {
        const int32_t bit0 = (int32_t)(j * 32) - (int32_t)sh;
        uint32_t mw;
        if (bit0 <= -32 || bit0 >= 64) mw = 0;
        else if (bit0 < 0) mw = (uint32_t)(m << (-bit0));
        else mw = (uint32_t)(m >> bit0);
        vf.at(dst + j) = __builtin_addc(cst(k.gconsts)[s.p[0] + j], mw, cy, &cy);
      }
      break;
    }
    case MG_GEN_FIXED:
      for (uint32_t j = 0; j < L; j++) vf.at(dst + j) = cst(k.gconsts)[s.p[0] + j];
      break;
    case MG_GEN_MIXED: {
      const uint32_t h = grnd(ky, c, 0xFFFFu);
      if (alt == ALT_DICT) {
        const uint32_t e = ((h >> 16) * s.p[1]) >> 16;
        if (L == 8) {
          uint32_t x[8];
#pragma unroll
          for (uint32_t j = 0; j < 8; j++) x[j] = gword(k, s.p[0] + e * 8 + j);
          sta8(vf, dst, x);
        } else {
          for (uint32_t j = 0; j < L; j++) vf.at(dst + j) = gword(k, s.p[0] + e * L + j);
        }
      } else {  // SMALL / UNIFORM
        const bool narrow = width <= MG_GEN_NARROW_BITS;
        const uint32_t bits = alt == ALT_SMALL ? min(width, s.p[4] >> 16) : width;
        uint32_t u1 = 0, u2 = 0;  // raw limbs j-1, j-2 (GEN3 gext chain)
        for (uint32_t j = 0; j < L; j++) {
          const uint32_t lo = j * 32;
          uint32_t v = 0;
          if (lo < bits) {  // limbs past `bits` are zero, and no later limb needs their raw value
            v = narrow ? (j == 0 ? (h & 0xFFFFu) : 0u) : j < 2 ? grnd(ky, c, j) : gext(u1, u2, j);
            u2 = u1;
            u1 = v;
          }
          vf.at(dst + j) = lo >= bits ? 0u : (bits - lo >= 32 ? v : (v & ((1u << (bits - lo)) - 1u)));
        }
      }
      break;
    }
    default: {  // UNIFORM (and LAZY coordinates, which the program never reads)
      uint32_t u1 = 0, u2 = 0;
      for (uint32_t j = 0; j < L; j++) {
        const uint32_t v = j < 2 ? grnd(ky, c, j) : gext(u1, u2, j);
        vf.at(dst + j) = v;
        u2 = u1;
        u1 = v;
      }
      break;
    }
  }
}

// MIXED: per-lane delta on COPY/DICT, width mask, clamp; every kind: width mask, fixed bits
template <class VF>
__device__ __forceinline__ void gen_finish(const KArgs& k, const VF& vf, uint32_t dst, uint32_t c, uint32_t width,
                           const GKeys& ky, const GenSpec& s, uint32_t alt, uint32_t ws) {
  const uint32_t L = (width + 31) >> 5;
  if (MG_GEN_KIND(s.kind) == MG_GEN_MIXED) {
    if ((alt == ALT_COPY || alt == ALT_DICT) && (ws & 0xFFFFu) < s.p[5]) {
      const uint32_t h = grnd(ky, c, 0xFFFFu);
      const uint32_t mag = 1u + (h & 1u);
      const bool sub = (h >> 1) & 1u;
      const uint32_t a0 = sub ? 0u - mag : mag, ah = sub ? 0xFFFFFFFFu : 0u;  // +/-mag sign-extended
      uint32_t cy = 0;
      if (L == 8) {
        uint32_t x[8];
        lda8(vf, dst, x);
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) x[j] = __builtin_addc(x[j], j ? ah : a0, cy, &cy);
        sta8(vf, dst, x);
      } else {
        for (uint32_t j = 0; j < L; j++) vf.at(dst + j) = __builtin_addc(vf.at(dst + j), j ? ah : a0, cy, &cy);
      }
    }
    vf.at(dst + L - 1) &= top_mask(width);
    if (s.p[6]) {  // clamp into [lo, lo + span)
      const auto* lo = cst(k.gconsts) + (s.p[6] - 1);
      const uint32_t span = lo[L];
      uint32_t br = 0, hi_or = 0, t0 = 0;
      for (uint32_t j = 0; j < L; j++) {
        const uint32_t t = __builtin_subc(vf.at(dst + j), lo[j], br, &br);
        if (j == 0) t0 = t;
        else hi_or |= t;
      }
      if (br || hi_or || (span && t0 >= span)) {
        const uint32_t v0 = vf.at(dst);
        const uint32_t off = span ? (uint32_t)(((uint64_t)v0 * span) >> 32) : v0;
        uint32_t cy = 0;
        for (uint32_t j = 0; j < L; j++) vf.at(dst + j) = __builtin_addc(lo[j], j ? 0u : off, cy, &cy);
      }
    }
  }
  vf.at(dst + L - 1) &= top_mask(width);
  if (const uint32_t fix = s.kind >> 8) {
    const auto* f = cst(k.gconsts) + (fix - 1);
    if (L == 8) {
      uint32_t x[8];
      lda8(vf, dst, x);
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) x[j] = (x[j] & ~f[j]) | f[8 + j];
      sta8(vf, dst, x);
    } else {
      for (uint32_t j = 0; j < L; j++) vf.at(dst + j) = (vf.at(dst + j) & ~f[j]) | f[L + j];
    }
  }
}

// Final value of coordinate c.  A MIXED COPY is the source's final value; the chain
// c -> p3 -> ... ends at the first link whose group choice is not COPY (sources have
// smaller indices, so it ends; parse_gen bounds its static length).  The root is
// generated, then every link's finish is applied from the root back to c.
template <class VF>
__device__ __forceinline__ void gen_coord(const KArgs& k, const VF& vf, uint32_t dst, uint32_t c, uint32_t width, const GKeys& ky) {
  uint32_t m = 0, root = c;
  GenSpec s = ld_spec(k, c);
  uint32_t ws = 0, alt = ALT_NONE;
  for (;;) {
    alt = ALT_NONE;
    if (MG_GEN_KIND(s.kind) != MG_GEN_MIXED) break;
    ws = gwsel(ky, root);
    alt = mixed_alt(s, ws);
    if (alt != ALT_COPY) break;
    root = s.p[3];
    s = ld_spec(k, root);
    m++;
  }
  gen_base(k, vf, dst, root, width, ky, s, alt);
  gen_finish(k, vf, dst, root, width, ky, s, alt, ws);
  while (m-- > 0) {  // link m: m steps from c
    uint32_t l = c;
    for (uint32_t t = 0; t < m; t++) l = ld_spec(k, l).p[3];
    const GenSpec sl = ld_spec(k, l);
    gen_finish(k, vf, dst, l, width, ky, sl, ALT_COPY, gwsel(ky, l));
  }
}

// ---------------------------------------------------------------------------
// value-file helpers
// ---------------------------------------------------------------------------
template <class VF>
__device__ __forceinline__ void write_masked(const VF& vf, uint32_t dst, uint32_t L, uint32_t width) {
  vf.at(dst + L - 1) &= top_mask(width);
}

template <class VF>
__device__ __forceinline__ W8 ld8(const VF& vf, uint32_t off, uint32_t L) {
  W8 x;
#pragma unroll
  for (int i = 0; i < 8; i++) x.w[i] = (uint32_t)i < L ? vf.at(off + i) : 0u;
  return x;
}

template <class VF>
__device__ __forceinline__ void st8(const VF& vf, uint32_t off, uint32_t L, const W8& x) {
#pragma unroll
  for (int i = 0; i < 8; i++)
    if ((uint32_t)i < L) vf.at(off + i) = x.w[i];
}

// 32 bits of value (slot off, width w) starting at bit position p (zero beyond w)
template <class VF>
__device__ __forceinline__ uint32_t bits32(const VF& vf, uint32_t off, uint32_t w, uint32_t p) {
  if (p >= w) return 0u;
  const uint32_t L = (w + 31) >> 5;
  const uint32_t q = p >> 5, r = p & 31u;
  const uint32_t lo = vf.at(off + q);
  const uint32_t hi = (q + 1 < L) ? vf.at(off + q + 1) : 0u;
  return r ? ((lo >> r) | (hi << (32 - r))) : lo;
}

template <class VF>
__device__ __forceinline__ uint32_t keccak_byte(const VF& vf, uint32_t off, uint32_t len, uint32_t m) {
  // message byte m (big-endian value of 8*len bits)
  const uint32_t bitpos = 8u * (len - 1u - m);
  return (vf.at(off + (bitpos >> 5)) >> (bitpos & 31u)) & 0xFFu;
}

template <class VF>
__device__ __forceinline__ void do_keccak(const VF& vf, const Instr& in) {
  uint64_t st[25];
#pragma unroll
  for (int i = 0; i < 25; i++) st[i] = 0;
  const uint32_t len = in.p0;
  const uint32_t nblocks = len / 136u + 1u;
  for (uint32_t b = 0; b < nblocks; b++) {
    for (uint32_t t = 0; t < 17; t++) {
      uint64_t lane = 0;
      for (uint32_t k = 0; k < 8; k++) {
        const uint32_t m = b * 136u + t * 8u + k;
        uint32_t byte = m < len ? keccak_byte(vf, in.a, len, m) : 0u;
        if (m == len) byte |= 0x01u;
        if (m == nblocks * 136u - 1u) byte |= 0x80u;
        lane |= (uint64_t)byte << (8 * k);
      }
      // st[t] ^= lane with a compile-time index (t is uniform; unrolled select)
#pragma unroll
      for (int i = 0; i < 17; i++)
        if ((uint32_t)i == t) st[i] ^= lane;
    }
    keccak_f1600(st);
  }
  // value limb j = bswap32(digest dword 7-j); digest dword 2t / 2t+1 = low / high of st[t]
  uint32_t dw[8];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    dw[2 * t] = (uint32_t)st[t];
    dw[2 * t + 1] = (uint32_t)(st[t] >> 32);
  }
#pragma unroll
  for (int j = 0; j < 8; j++) vf.at(in.dst + j) = __builtin_bswap32(dw[7 - j]);
}

// ---------------------------------------------------------------------------
// interpreter
// ---------------------------------------------------------------------------
// Per-limb loops run fully unrolled for the two widths that dominate LASER queries
// (L = 8: 256-bit words; L = 1: Bools, bytes, <= 32-bit values): the value-file
// offsets then fold into the ds_read/ds_write immediates and the limb control leaves
// the scalar unit (a rolled loop costs ~6 SALU + a branch per limb).
#define MG_LIMBS(L, BODY)                        \
  do {                                           \
    if ((L) == 8) {                              \
      _Pragma("unroll") for (uint32_t j = 0; j < 8; j++) { BODY }  \
    } else if ((L) == 1) {                       \
      const uint32_t j = 0;                      \
      { BODY }                                   \
    } else {                                     \
      for (uint32_t j = 0; j < (L); j++) { BODY } \
    }                                            \
  } while (0)

// EQ / ULT / ULE / SLT / SLE of the width-wa values in slots a and b (0 or 1)
template <class VF>
__device__ __forceinline__ uint32_t compare(const VF& vf, uint32_t op, uint32_t a, uint32_t b, uint32_t wa) {
  const uint32_t La = (wa + 31) >> 5;
  if (op == K_EQ) {
    uint32_t d = 0;
    MG_LIMBS(La, d |= vf.at(a + j) ^ vf.at(b + j););
    return d == 0;
  }
  // a - b borrow chain; for signed compare flip the sign bits first
  const uint32_t sflip = (op == K_SLT || op == K_SLE) ? (1u << ((wa - 1) & 31)) : 0u;
  uint32_t br = 0, nz = 0;
  MG_LIMBS(La, {
    const uint32_t f = j == La - 1 ? sflip : 0u;
    nz |= __builtin_subc(vf.at(a + j) ^ f, vf.at(b + j) ^ f, br, &br);
  });
  const bool lt = br != 0;
  const bool le = lt || nz == 0;
  return (op == K_ULT || op == K_SLT) ? (uint32_t)lt : (uint32_t)le;
}

// TIER: the handlers a program needs.  kTierLight: no MUL/DIV/REM/shift/EXP/UMUL_NOOVF/KECCAK
// (most LASER queries; 47 VGPRs); kTierMid adds MUL, UMUL_NOOVF and the shifts (the overflow
// checks of arithmetic); kTierHeavy adds division, EXP and Keccak, whose 256-bit temporaries
// hold ~220 VGPRs (two waves per SIMD).  Leaving handlers out lets more waves hide the LDS and
// scalar-load latency.
// One wave evaluates KG groups of 64 candidates per program pass: every dispatched instruction (its
// scalar fetch, decode and jump) runs its handler once per group, on the group's slice of the value
// file (VFG: slot-major, [slot][group][lane]).  verdict[g], i[g], key[g], active[g] are per group.
template <class VF, int KG>
struct VFG {
  VF f;
  uint32_t g;
  __device__ __forceinline__ uint32_t& at(uint32_t w) const { return f.at(w * KG + g); }
};

#define MG_FOR_G(...)                                   \
  _Pragma("unroll") for (uint32_t g = 0; g < (uint32_t)KG; g++) { \
    const VFG<VF, KG> vf{vf0, g};                       \
    __VA_ARGS__                                         \
  }

template <class VF, int MODE, int TIER, int KG>
__device__ __forceinline__ void run_program(const KArgs& k, const VF& vf0, const uint64_t* i, const GKeys* key,
                                            bool early, const bool* active, uint32_t* verdict) {
_Pragma("unroll")
  for (int g = 0; g < KG; g++) verdict[g] = 1;
  const uint32_t n_instr = k.n_instr;
  // the next instruction's scalar load is issued before this one executes, so its latency
  // overlaps this instruction's LDS traffic instead of adding to it (the code buffer has
  // one padding record after the last instruction)
  Instr nx = ld_instr(k, k.pc0);
  bool stop = false;
  for (uint32_t pc = k.pc0; pc < n_instr && !stop; pc++) {
    const Instr in = nx;
    nx = ld_instr(k, pc + 1);
    const uint32_t W = in.wd;
    const uint32_t L = (W + 31) >> 5;
    switch (in.op) {
      case K_CONST: {
        const auto* c = cst(k.consts) + in.p0;
        MG_FOR_G(MG_LIMBS(L, vf.at(in.dst + j) = c[j];););
        break;
      }
      case K_COORD: {
        if (MODE == MODE_EVAL) {
          MG_FOR_G(MG_LIMBS(L, vf.at(in.dst + j) = k.soa[(uint64_t)(in.p1 + j) * k.count + i[g]];););
        } else {
          MG_FOR_G(gen_coord<VFG<VF, KG>>(k, vf, in.dst, in.p0, W, key[g]););
        }
        break;
      }
      case K_COPY: {
        MG_FOR_G({
          if (L == 8) {
            uint32_t x[8];
            lda8(vf, in.a, x);
            sta8(vf, in.dst, x);
          } else {
            MG_LIMBS(L, vf.at(in.dst + j) = vf.at(in.a + j););
          }
        });
        break;
      }
      case K_ADD:
      case K_SUB: {
        MG_FOR_G({
          if (L == 8) {
            uint32_t x[8], y[8], r[8], c = 0;
            lda8(vf, in.a, x);
            lda8(vf, in.b, y);
            if (in.op == K_ADD) {
_Pragma("unroll")
              for (int j = 0; j < 8; j++) r[j] = __builtin_addc(x[j], y[j], c, &c);
            } else {
_Pragma("unroll")
              for (int j = 0; j < 8; j++) r[j] = __builtin_subc(x[j], y[j], c, &c);
            }
            r[7] &= top_mask(W);
            sta8(vf, in.dst, r);
          } else {
            uint32_t c = 0;
            if (in.op == K_ADD) {
              MG_LIMBS(L, vf.at(in.dst + j) = __builtin_addc(vf.at(in.a + j), vf.at(in.b + j), c, &c););
            } else {
              MG_LIMBS(L, vf.at(in.dst + j) = __builtin_subc(vf.at(in.a + j), vf.at(in.b + j), c, &c););
            }
            write_masked(vf, in.dst, L, W);
          }
        });
        break;
      }
      case K_NEG: {
        MG_FOR_G({
          if (L == 8) {
            uint32_t x[8], r[8], c = 0;
            lda8(vf, in.a, x);
_Pragma("unroll")
            for (int j = 0; j < 8; j++) r[j] = __builtin_subc(0u, x[j], c, &c);
            r[7] &= top_mask(W);
            sta8(vf, in.dst, r);
          } else {
            uint32_t c = 0;
            MG_LIMBS(L, vf.at(in.dst + j) = __builtin_subc(0u, vf.at(in.a + j), c, &c););
            write_masked(vf, in.dst, L, W);
          }
        });
        break;
      }
      case K_AND:
      case K_OR:
      case K_XOR: {
        MG_FOR_G({
          if (L == 8) {
            uint32_t x[8], y[8], r[8];
            lda8(vf, in.a, x);
            lda8(vf, in.b, y);
_Pragma("unroll")
            for (int j = 0; j < 8; j++) r[j] = in.op == K_AND ? (x[j] & y[j]) : in.op == K_OR ? (x[j] | y[j]) : (x[j] ^ y[j]);
            sta8(vf, in.dst, r);
          } else if (in.op == K_AND) {
            MG_LIMBS(L, vf.at(in.dst + j) = vf.at(in.a + j) & vf.at(in.b + j););
          } else if (in.op == K_OR) {
            MG_LIMBS(L, vf.at(in.dst + j) = vf.at(in.a + j) | vf.at(in.b + j););
          } else {
            MG_LIMBS(L, vf.at(in.dst + j) = vf.at(in.a + j) ^ vf.at(in.b + j););
          }
        });
        break;
      }
      case K_NOT:
        MG_FOR_G({
          if (L == 8) {
            uint32_t x[8];
            lda8(vf, in.a, x);
_Pragma("unroll")
            for (int j = 0; j < 8; j++) x[j] = ~x[j];
            x[7] &= top_mask(W);
            sta8(vf, in.dst, x);
          } else {
            MG_LIMBS(L, vf.at(in.dst + j) = ~vf.at(in.a + j););
            write_masked(vf, in.dst, L, W);
          }
        });
        break;
      case K_ITE: {
        MG_FOR_G({
          const bool c = vf.at(in.a) != 0;
          if (L == 8) {
            uint32_t x[8], y[8];
            lda8(vf, in.b, x);
            lda8(vf, in.c, y);
_Pragma("unroll")
            for (int j = 0; j < 8; j++) x[j] = c ? x[j] : y[j];
            sta8(vf, in.dst, x);
          } else {
            MG_LIMBS(L, vf.at(in.dst + j) = c ? vf.at(in.b + j) : vf.at(in.c + j););
          }
        });
        break;
      }
      case K_EQ: {
        const uint32_t La = (in.p1 + 31) >> 5;
        MG_FOR_G({
          uint32_t d = 0;
          MG_LIMBS(La, d |= vf.at(in.a + j) ^ vf.at(in.b + j););
          vf.at(in.dst) = d == 0;
        });
        break;
      }
      case K_ULT:
      case K_ULE:
      case K_SLT:
      case K_SLE:
        MG_FOR_G(vf.at(in.dst) = compare(vf, in.op, in.a, in.b, in.p1););
        break;
      case K_ASSERT_CMP: {
        // a compare whose one use was this assert (program.cpp: fuse_asserts)
        uint64_t any = 0;
        MG_FOR_G({
          verdict[g] &= compare(vf, in.p0 & 0xFFu, in.a, in.b, in.p1) ^ (in.p0 >> 8);
          any |= __ballot(verdict[g] != 0);
        });
        if (early && __builtin_amdgcn_readfirstlane((uint32_t)(any != 0ull)) == 0u) stop = true;
        break;
      }
      case K_CONCAT: {
        // dst = a:b, width(b) = p1
        const uint32_t wb = in.p1, wa = W - wb;
        MG_FOR_G({
          if (L == 8) {  // every limb computed (loads only) before the stores
            uint32_t r[8];
_Pragma("unroll")
            for (uint32_t j = 0; j < 8; j++) {
              const uint32_t p = j * 32;
              uint32_t v = bits32(vf, in.b, wb, p);
              if (p + 32 > wb) {
                v |= (p >= wb) ? bits32(vf, in.a, wa, p - wb) : (bits32(vf, in.a, wa, 0) << (wb - p));
              }
              r[j] = v;
            }
            r[7] &= top_mask(W);
            sta8(vf, in.dst, r);
          } else {
            for (uint32_t j = 0; j < L; j++) {
              const uint32_t p = j * 32;
              uint32_t v = bits32(vf, in.b, wb, p);
              if (p + 32 > wb) {
                v |= (p >= wb) ? bits32(vf, in.a, wa, p - wb) : (bits32(vf, in.a, wa, 0) << (wb - p));
              }
              vf.at(in.dst + j) = v;
            }
            write_masked(vf, in.dst, L, W);
          }
        });
        break;
      }
      case K_EXTRACT: {
        MG_FOR_G({
          if (L == 1) {
            vf.at(in.dst) = bits32(vf, in.a, in.p1, in.p0) & top_mask(W);
          } else if (L == 8) {
            uint32_t r[8];
_Pragma("unroll")
            for (uint32_t j = 0; j < 8; j++) r[j] = bits32(vf, in.a, in.p1, in.p0 + j * 32);
            r[7] &= top_mask(W);
            sta8(vf, in.dst, r);
          } else {
            for (uint32_t j = 0; j < L; j++) vf.at(in.dst + j) = bits32(vf, in.a, in.p1, in.p0 + j * 32);
            write_masked(vf, in.dst, L, W);
          }
        });
        break;
      }
      case K_ZEXT:
      case K_SEXT: {
        const uint32_t wa = in.p1, La = (wa + 31) >> 5;
        const uint32_t tm = top_mask(wa);
        MG_FOR_G({
          uint32_t fill = 0;
          if (in.op == K_SEXT) fill = ((vf.at(in.a + La - 1) >> ((wa - 1) & 31)) & 1u) ? 0xFFFFFFFFu : 0u;
          if (L == 8) {
            uint32_t r[8];
_Pragma("unroll")
            for (uint32_t j = 0; j < 8; j++) {
              uint32_t v = fill;
              if (j < La) {
                v = vf.at(in.a + j);
                if (j == La - 1) v = (v & tm) | (fill & ~tm);
              }
              r[j] = v;
            }
            r[7] &= top_mask(W);
            sta8(vf, in.dst, r);
          } else {
            MG_LIMBS(L, {
              uint32_t v = fill;
              if (j < La) {
                v = vf.at(in.a + j);
                if (j == La - 1) v = (v & tm) | (fill & ~tm);
              }
              vf.at(in.dst + j) = v;
            });
            write_masked(vf, in.dst, L, W);
          }
        });
        break;
      }
      case K_MUL: {
        if constexpr (TIER >= kTierMid) {
          MG_FOR_G({
            W8 r = mul8(ld8(vf, in.a, L), ld8(vf, in.b, L));
            canon8(r, W);
            st8(vf, in.dst, L, r);
          });
        }
        break;
      }
      case K_UMUL_NOOVF: {
        if constexpr (TIER >= kTierMid) {
          const uint32_t wa = in.p1, La = (wa + 31) >> 5;
          MG_FOR_G(vf.at(in.dst) = umul_noovf8(ld8(vf, in.a, La), ld8(vf, in.b, La), wa););
        }
        break;
      }
      case K_UDIV: if constexpr (TIER >= kTierHeavy) { MG_FOR_G(st8(vf, in.dst, L, bv_udiv(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_UREM: if constexpr (TIER >= kTierHeavy) { MG_FOR_G(st8(vf, in.dst, L, bv_urem(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_SDIV: if constexpr (TIER >= kTierHeavy) { MG_FOR_G(st8(vf, in.dst, L, bv_sdiv(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_SREM: if constexpr (TIER >= kTierHeavy) { MG_FOR_G(st8(vf, in.dst, L, bv_srem(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_SMOD: if constexpr (TIER >= kTierHeavy) { MG_FOR_G(st8(vf, in.dst, L, bv_smod(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_SHL: if constexpr (TIER >= kTierMid) { MG_FOR_G(st8(vf, in.dst, L, bv_shl(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_LSHR: if constexpr (TIER >= kTierMid) { MG_FOR_G(st8(vf, in.dst, L, bv_lshr(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_ASHR: if constexpr (TIER >= kTierMid) { MG_FOR_G(st8(vf, in.dst, L, bv_ashr(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_EXP: if constexpr (TIER >= kTierHeavy) { MG_FOR_G(st8(vf, in.dst, L, bv_exp(ld8(vf, in.a, L), ld8(vf, in.b, L), W));); } break;
      case K_LOOKUP: {
        const uint32_t Lk = (in.b + 31) >> 5;
        MG_FOR_G({
          uint32_t src = in.p0;
          bool found = false;
          for (uint32_t p = 0; p < in.c; p++) {
            const uint32_t ko = cst(k.aux)[in.p1 + 2 * p], vo = cst(k.aux)[in.p1 + 2 * p + 1];
            uint32_t d = 0;
            MG_LIMBS(Lk, d |= vf.at(in.a + j) ^ vf.at(ko + j););
            const bool hit = !found && d == 0;
            src = hit ? vo : src;
            found = found || hit;
          }
          // src differs per lane: gather the limbs from the selected slot
          if (L == 8) {
            uint32_t x[8];
            lda8(vf, src, x);
            sta8(vf, in.dst, x);
          } else {
            MG_LIMBS(L, vf.at(in.dst + j) = vf.at(src + j););
          }
        });
        break;
      }
      case K_KECCAK: {
        if (in.a == MG_NONE) {
          // keccak256("") — the constant of keccak_function_manager.py:75-81
          MG_FOR_G(for (uint32_t j = 0; j < 8; j++) vf.at(in.dst + j) = kEmptyKeccak[j];);
        } else if constexpr (TIER >= kTierHeavy) {
          MG_FOR_G(do_keccak(vf, in););
        }
        break;
      }
      case K_ASSERT: {
        // every lane of every group failed: stop (verdicts are 0 everywhere).  A loop flag, not a
        // return: a second loop exit made the compiler keep pc in a VGPR (vector address math +
        // readfirstlane per fetch); readfirstlane makes the flag's uniformity explicit
        uint64_t any = 0;
        MG_FOR_G({
          verdict[g] &= vf.at(in.a);
          any |= __ballot(verdict[g] != 0);
        });
        if (early && __builtin_amdgcn_readfirstlane((uint32_t)(any != 0ull)) == 0u) stop = true;
        break;
      }
      case K_WATCH: {
        if (MODE != MODE_SEARCH && k.watch) {
          MG_FOR_G({
            if (active[g])
              for (uint32_t j = 0; j < L; j++) k.watch[(uint64_t)(in.p0 + j) * k.count + i[g]] = vf.at(in.a + j);
          });
        } else if (MODE == MODE_SEARCH && k.watch) {
          // capture launch (one group per block, KG = 1): every lane's watch rows, [block][row][lane],
          // so the first hit's model is read back without a second program pass
          const VFG<VF, KG> vf{vf0, 0};
          uint32_t* w = k.watch + ((uint64_t)blockIdx.x * k.watch_words + in.p0) * kWave + threadIdx.x;
          for (uint32_t j = 0; j < L; j++) w[(uint64_t)j * kWave] = vf.at(in.a + j);
        }
        break;
      }
      default:
        break;
    }
  }
}

// one lane's column of a capture block: dst[r] = src[r * 64] (mg_search model read-back)
__global__ void __launch_bounds__(256) k_gather_rows(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                      uint32_t rows) {
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  if (r < rows) dst[r] = src[(uint64_t)r * kWave];
}

template <class VF, int MODE, int TIER, int KG>
__global__ void __launch_bounds__(kWave) k_run(KArgs k) {
  VF vf0(mg_lds, k);
  // the generator constants into LDS behind the value file (one wave per block: its own later
  // reads see the writes, LDS runs a wave's operations in order)
  if (MODE != MODE_EVAL && k.lds_g != kNoLds)
    for (uint32_t i = threadIdx.x; i < k.n_gconsts; i += kWave) mg_lds[k.lds_g + i] = cst(k.gconsts)[i];
  // EVAL sweeps rows [0, count); GEN / SEARCH sweep the aligned 64-index groups that
  // cover [start, start + count), one group per wave (the GEN3 group key is per wave)
  const uint64_t a0 = (MODE == MODE_EVAL) ? 0ull : (k.start & ~63ull);
  const uint64_t end = k.start + k.count;
  const uint64_t total = (MODE == MODE_EVAL) ? k.count : (end - a0);
  // KG groups per wave per pass (run_program): a wave's pass covers KG * 64 consecutive indices
  const uint64_t step = (uint64_t)gridDim.x * kWave * KG;
  const bool early = (MODE == MODE_SEARCH) && (k.flags & MG_SEARCH_EARLY_EXIT);
  uint64_t wave_best = ~0ull, wave_hits = 0;  // wave-uniform; published once per wave
  // idx & 63 == threadIdx.x & 63 below (a0 and base are multiples of 64): the lane half of
  // the GEN3 lane key is fixed per thread
  const uint64_t lk = (MODE == MODE_EVAL) ? 0ull : gen_lane_key(threadIdx.x & 63u, k.sk);
  // Warm the scalar cache with the program and the generator specs, 64-byte lines eight loads at a
  // time: a wave reads them with dependent scalar loads, one instruction (32 B) or spec ahead, so a
  // cold cache costs it an L2 round trip every other instruction — the floor of an easy query's time
  // to first model, which one wave's pass over the program is.
  if (k.flags & kFlagPrefetch) {
    uint32_t acc = 0;
    auto warm = [&acc](const uint32_t* base, uint32_t lines) {
      const auto* b = cst(base);
      for (uint32_t l = 0; l < lines; l += 8) {
        uint32_t x[8];
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = (l + q < lines) ? b[16u * (l + q)] : 0u;
#pragma unroll
        for (int q = 0; q < 8; q++) acc ^= x[q];
      }
    };
    warm((const uint32_t*)k.code, min((k.n_instr + 2u) / 2u, 512u));
    if (MODE != MODE_EVAL && k.specs) warm((const uint32_t*)k.specs, min((k.n_specs + 1u) / 2u, 512u));
    if (acc == 0x5EED1E55u && k.count == ~0ull) k.hits[0] = acc;  // never true: keeps the loads
  }
  // the hoisted literals: their slots are never reused, so once per thread is enough
  for (uint32_t pc = 0; pc < k.pc0; pc++) {
    const Instr in = ld_instr(k, pc);
    const uint32_t L = (in.wd + 31) >> 5;
    const auto* c = cst(k.consts) + in.p0;
    MG_FOR_G(MG_LIMBS(L, vf.at(in.dst + j) = c[j];););
  }
  for (uint64_t base = (uint64_t)blockIdx.x * kWave * KG; base < total; base += step) {
    bool active[KG];
    uint64_t i[KG];
    GKeys key[KG];
#pragma unroll
    for (int g = 0; g < KG; g++) {
      const uint64_t off = base + (uint64_t)g * kWave + threadIdx.x;
      const uint64_t idx = a0 + off;  // candidate index (GEN / SEARCH)
      active[g] = (MODE == MODE_EVAL) ? off < total : (idx >= k.start && idx < end);
      // EVAL: SoA row; GEN: output row (only written by active lanes)
      i[g] = (MODE == MODE_EVAL) ? (active[g] ? off : total - 1) : (idx - k.start);
    }
    uint64_t cur_u = ~0ull;  // the hit word as this group starts (early exit only)
    if (early) {
      // every candidate below the current first hit is still evaluated, so the
      // final minimum is exact; waves entirely above it stop
      const unsigned long long cur = read_first_hit(k.first_hit, k.flags);
      // readfirstlane returns int: widen through uint32_t, or a low word with bit 31 set would
      // sign-extend over the high word
      cur_u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cur >> 32)) << 32) |
              (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cur);
      if (a0 + base >= cur_u) break;
    }
    // each group's key from its base (a0 + base + 64 g, a multiple of 64: idx >> 6 is the same for
    // every lane), so the compiler sees G as wave-uniform: the MIXED alternatives are scalar branches
    // and the generator specs scalar loads (from idx, G looked per-lane: divergent branches, vector loads)
#pragma unroll
    for (int g = 0; g < KG; g++) key[g] = MODE != MODE_EVAL ? gen_keys_lk(a0 + base + (uint64_t)g * kWave, lk, k.sg) : GKeys{};
    uint32_t v[KG];
    run_program<VF, MODE, TIER, KG>(k, vf0, i, key, early, active, v);
#pragma unroll
    for (int g = 0; g < KG; g++) {
      v[g] = active[g] ? v[g] : 0u;
      if (MODE == MODE_SEARCH) {
        const unsigned long long m = __ballot(v[g] != 0);
        if (m) {
          const uint64_t first = a0 + base + (uint64_t)g * kWave + (uint64_t)(__ffsll((long long)m) - 1);
          wave_hits += (uint64_t)__popcll(m);
          if (first < wave_best) {
            wave_best = first;
            // (a hit at or above the word read as the group started cannot lower it: no atomic)
            if (early && threadIdx.x == 0 && first < cur_u) {
              atomicMin(k.first_hit, (unsigned long long)first);
              publish_peers(k.first_hit, (unsigned long long)first);
            }
          }
        }
      } else if (active[g]) {
        k.verdict[i[g]] = (uint8_t)v[g];
      }
    }
  }
  if (MODE == MODE_SEARCH && threadIdx.x == 0) {
    // a first hit that cannot lower the current minimum is not published; the count goes to the
    // block's stripe (kHitStripes)
    if (wave_best != ~0ull &&
        wave_best < read_first_hit(k.first_hit, k.flags))
      atomicMin(k.first_hit, (unsigned long long)wave_best);
    if (wave_hits) atomicAdd(k.hits + kHitStride * (1u + (blockIdx.x % kHitStripes)) - 1u, (unsigned long long)wave_hits);
  }
}

// batched concrete Keccak-256: one lane per message
__global__ void __launch_bounds__(256) k_keccak(const uint8_t* msgs, const uint64_t* offs, const uint32_t* lens,
                                                 uint64_t n, uint8_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* m = msgs + offs[i];
  const uint32_t len = lens[i];
  uint64_t st[25];
#pragma unroll
  for (int q = 0; q < 25; q++) st[q] = 0;
  const uint32_t nblocks = len / 136u + 1u;
  for (uint32_t b = 0; b < nblocks; b++) {
#pragma unroll
    for (int t = 0; t < 17; t++) {
      uint64_t lane = 0;
      for (int kb = 0; kb < 8; kb++) {
        const uint32_t pos = b * 136u + t * 8u + kb;
        uint32_t byte = pos < len ? m[pos] : 0u;
        if (pos == len) byte |= 0x01u;
        if (pos == nblocks * 136u - 1u) byte |= 0x80u;
        lane |= (uint64_t)byte << (8 * kb);
      }
      st[t] ^= lane;
    }
    keccak_f1600(st);
  }
#pragma unroll
  for (int t = 0; t < 4; t++) {
#pragma unroll
    for (int kb = 0; kb < 8; kb++) out[i * 32 + t * 8 + kb] = (uint8_t)(st[t] >> (8 * kb));
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
thread_local std::string g_err;

struct DevProgram {
  Lowered low;
  std::string src;  // the program bytes (key of the specialisation cache)
  int tier = 2;  // interpreter variant: kTierLight / kTierMid / kTierHeavy (run_program)
  bool uploaded = false;
  void* buf = nullptr;  // pooled device buffer holding the four arrays below
  size_t cap = 0;
  Instr* d_code = nullptr;
  uint32_t* d_consts = nullptr;
  uint32_t* d_aux = nullptr;
  uint32_t* d_coord_width = nullptr;
  bool lds = false;
};

struct Engine;
static void pool_put(Engine& e, void* ptr, size_t cap);

// specialisations of one (program, generator) pair, shared through the cache.  On the primary
// device they stay uploaded with the cache entry (`dev`): LASER re-asks constraint sets, and a
// repeat's mg_gen_load then makes no copy to the device (three synchronous copies, ~50 us, were
// a quarter of a warm query's time to first model).  A generator loaded from the entry borrows
// these buffers (DevGen::borrowed); they go back to the pool when the last holder lets go.
struct SpecSet {
  DevProgram search, watch;  // .low: the specialised programs
  std::shared_ptr<Lowered> model;  // watch list only, asserts dropped: built on the first hit
  Engine* dev = nullptr;     // the device the buffers below live on (nullptr: not uploaded)
  void* gbuf = nullptr;      // generator specs | constants
  size_t gcap = 0;
  GenSpec* d_specs = nullptr;
  uint32_t* d_consts = nullptr;
  ~SpecSet();
};

struct DevGen {
  uint64_t prog = 0;
  std::shared_ptr<SpecSet> set;   // (primary) where the model-only variant is cached
  DevProgram spec_model;          // that variant, uploaded on the first model read-back
  std::vector<GenSpec> specs;     // host copies: the JIT specialises on them
  std::vector<uint32_t> consts;
  GenSpec* d_specs = nullptr;
  uint32_t* d_consts = nullptr;
  DevProgram spec;                // the program specialised for this generator (what searches run)
  DevProgram spec_watch;          // the same with the watch list (model read-back, mg_eval_generated)
  void* gbuf = nullptr;           // pooled buffer behind d_specs / d_consts
  size_t gcap = 0;
  bool borrowed = false;          // spec / spec_watch / d_specs / d_consts are `set`'s (not freed here)
};

// a loaded JIT module shared by the code cache and the kernels handed out from it: unloaded
// when the last holder lets go
struct ModHold {
  hipModule_t mod = nullptr;
  explicit ModHold(hipModule_t m) : mod(m) {}
  ~ModHold() {
    if (mod) (void)hipModuleUnload(mod);
  }
};

struct DevJit {
  std::vector<char> code;  // the code object (loaded again on the node's other devices)
  hipModule_t mod = nullptr;
  std::shared_ptr<ModHold> hold;  // set: `mod` belongs to it (primary device, code cache)
  hipFunction_t fsearch = nullptr, feval = nullptr, fgen = nullptr;
  uint64_t prog = 0, gen = 0;
  int nb_search = 1, nb_eval = 1;
  double compile_ms = 0;
  bool asm_tier = false;  // the first tier's kernels (jit_asm.cpp): an eval launch takes n < 2^30
  bool tiled = false;     // eval kernel compiled for the tiled SoA (MG_JIT_SOA_TILED)
  // candidates per workgroup of a loop-free eval kernel (the first tier's `solo` read-backs: one
  // 64-candidate group per workgroup, launched ceil(n / 64) wide); 0: the kernel loops over groups;
  // -1: not read yet from the code object (code_object_info, mgj_meta_eval_cpb)
  int eval_cpb = -1;
};

// unload (or let go of) a JIT kernel's module
static void release_jit(DevJit& j) {
  if (j.hold) j.hold.reset();
  else if (j.mod) (void)hipModuleUnload(j.mod);
  j.mod = nullptr;
}

// compiled code objects by source text, least recently used first out (MYTHGPU_JIT_CACHE
// entries, default 64): JIT sources embed the query, so this only serves repeats
struct CodeCache {
  struct Entry {
    std::string src;
    std::vector<char> code;
    // the module as loaded on the primary device, kept resident: a repeated query's kernel is
    // ready without a module load (hipModuleLoadData per repeat was most of a warm switch)
    std::shared_ptr<ModHold> hold;
    hipFunction_t fsearch = nullptr, feval = nullptr, fgen = nullptr;
    int nb_search = 1, nb_eval = 1;
  };
  std::list<Entry> lru;  // front = most recent
  std::unordered_multimap<size_t, std::list<Entry>::iterator> idx;
  size_t cap = 64;
  Entry* find_entry(const std::string& src) {
    const size_t h = std::hash<std::string>()(src);
    auto r = idx.equal_range(h);
    for (auto it = r.first; it != r.second; ++it)
      if (it->second->src == src) {
        lru.splice(lru.begin(), lru, it->second);
        return &*it->second;
      }
    return nullptr;
  }
  const std::vector<char>* find(const std::string& src) {
    Entry* en = find_entry(src);
    return en ? &en->code : nullptr;
  }
  const std::vector<char>* insert(const std::string& src, std::vector<char>&& code) {
    if (const auto* c = find(src)) return c;
    lru.push_front(Entry{src, std::move(code), nullptr});
    idx.emplace(std::hash<std::string>()(src), lru.begin());
    while (lru.size() > cap) {
      auto last = std::prev(lru.end());
      auto r = idx.equal_range(std::hash<std::string>()(last->src));
      for (auto it = r.first; it != r.second; ++it)
        if (it->second == last) {
          idx.erase(it);
          break;
        }
      lru.erase(last);
    }
    return &lru.front().code;
  }
};

// one JIT compile request: the inputs are copied at submission, so the caller may free
// the program / generator meanwhile (the result is then dropped)
struct JitTicket {
  enum State { PENDING, DONE, FAILED } state = PENDING;
  uint64_t prog = 0, gen = 0;
  uint32_t flags = 0;
  Lowered low;
  bool has_gen = false;
  std::vector<GenSpec> specs;
  std::vector<uint32_t> consts;
  bool cancelled = false;
  bool asm_fallback = false;  // the first tier was chosen by default (watch rows): O3 if it refuses
  bool auto_eval = false;     // verdict-only eval, no tier asked for: the worker picks (eval_tier_pick)
  std::unique_ptr<DevJit> ready;  // loaded module, handed to Engine::jits by the poll
  int rc = MG_OK;
  std::string err;
  std::chrono::steady_clock::time_point submitted = std::chrono::steady_clock::now();  // MYTHGPU_JIT_TIMING
};

struct Engine {
  std::mutex mu;
  std::unordered_map<uint64_t, std::unique_ptr<DevJit>> jits;
  CodeCache code_cache;
  // host-side results of the per-query passes, by input bytes (FIFO, `cache_cap` entries):
  // LASER re-asks the same constraint sets, and a repeat then skips lowering and the two
  // generator specialisations (mg_program_load / mg_gen_load)
  std::unordered_map<std::string, std::shared_ptr<Lowered>> lower_cache;
  std::unordered_map<std::string, std::shared_ptr<SpecSet>> spec_cache;
  std::deque<std::string> lower_order, spec_order;
  size_t cache_cap = 64;
  // compile thread: source emission, comgr and the module load run off the caller's thread
  // and never take `mu` (a search holds `mu` for its whole launch + sync, back to back), so
  // searches keep launching while a query's kernel compiles (mg_jit_compile_async).  `jit_mu`
  // guards the members below; lock order: mu before jit_mu.
  std::mutex jit_mu;
  // two compile threads (detached; never outlive the leaked Engine), one per queue: [0] the O3
  // kernels (clang + LLVM, ~140 ms), [1] the first tier (assembly, a few ms) — a first-tier request
  // never waits behind an O3 compile, not even a cancelled one still in the compiler
  int jit_workers = 0;
  bool jit_stop = false;
  std::deque<std::shared_ptr<JitTicket>> jit_queue[2];
  std::unordered_map<uint64_t, std::shared_ptr<JitTicket>> tickets;
  std::condition_variable jit_cv, jit_done_cv;
  // sources being compiled right now: a second request for one waits for the first's code object
  // (LASER re-asks a query while its first compile, cancelled with its search, still runs)
  std::unordered_set<std::string> jit_inflight;
  bool init = false;
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  int cu_count = 0, clock_mhz = 0;
  // the mask spans physical devices: hit buffers are fine-grained and launches read them with
  // system scope (MG_SEARCH_SYSTEM_SCOPE)
  bool sys_scope = false;
  uint64_t next_handle = 1;
  std::unordered_map<uint64_t, std::unique_ptr<DevProgram>> progs;
  std::unordered_map<uint64_t, std::unique_ptr<DevGen>> gens;
  unsigned long long* d_hit = nullptr;  // [0] first hit, [1] hit count
  uint32_t* d_capture = nullptr;         // watch-row capture of a one-group-per-block search
  size_t capture_bytes = 0;
  // pinned host staging: [0..1] the reset values, [2..3] the result (async copies on `stream`,
  // one event wait per call instead of two blocking hipMemcpy round trips)
  unsigned long long* h_hit = nullptr;
  uint32_t* h_watch1 = nullptr;  // pinned copy of d_watch1
  size_t h_watch1_words = 0;
  uint32_t* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  // device buffers of freed programs/generators, by capacity: a query's uploads reuse them
  // instead of paying hipMalloc (tens to hundreds of microseconds each) per query
  std::multimap<size_t, void*> pool;
  uint32_t* d_watch1 = nullptr;  // one candidate's watch rows (model read-back)
  size_t watch1_words = 0;
  uint8_t* d_ver1 = nullptr;
  // mg_jit_search_many: kManySlots hit buffers (kHitAlloc words each, no peers) and their pinned
  // armed image / read-back, and kManyStreams streams the launches round-robin over (created on first use)
  unsigned long long* d_hitmany = nullptr;
  unsigned long long* h_hitmany = nullptr;
  hipStream_t xs[4] = {};
  hipEvent_t xev[4] = {};
  mg_stats_t stats{};
  uint64_t refused_base = 0;  // jit_refused_total() at the last mg_stats_reset
};

Engine& E() {
  // never destroyed: the detached JIT compile thread may still hold it at process exit
  static Engine* e = new Engine;
  return *e;
}

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t _e = (x);                                                           \
    if (_e != hipSuccess) {                                                        \
      g_err = std::string(#x) + ": " + hipGetErrorString(_e);                      \
      return MG_E_HIP;                                                             \
    }                                                                              \
  } while (0)

// The engine's primary device made current on the calling thread.  The z3 race calls the
// engine from two threads (the search on the GPU worker, mg_keccak256 from LASER's thread) and
// only the thread that ran mg_init had the device set: with MYTHGPU_DEVICE / LOCAL_RANK != 0
// the other one's hipMallocs landed on GPU 0 while its kernels ran on e.stream of GPU k.
// Every entry point that touches the device takes one after the engine lock.
struct OnDevice {
  explicit OnDevice(const Engine& e) {
    int d = -1;
    if (e.device >= 0 && (hipGetDevice(&d) != hipSuccess || d != e.device)) (void)hipSetDevice(e.device);
  }
};

static int set_err(int code, const std::string& m) {
  g_err = m;
  return code;
}

template <class T>
static int upload(T** d, const T* h, size_t n) {
  *d = nullptr;
  if (n == 0) n = 1;
  HIPCHK(hipMalloc((void**)d, n * sizeof(T)));
  if (h) HIPCHK(hipMemcpy(*d, h, n * sizeof(T), hipMemcpyHostToDevice));
  return MG_OK;
}

static int pool_get(Engine& e, size_t bytes, void** ptr, size_t* cap) {
  size_t c = 4096;
  while (c < bytes) c <<= 1;
  auto it = e.pool.find(c);
  if (it != e.pool.end()) {
    *ptr = it->second;
    e.pool.erase(it);
  } else {
    HIPCHK(hipMalloc(ptr, c));
  }
  *cap = c;
  return MG_OK;
}

static void pool_put(Engine& e, void* ptr, size_t cap) {
  if (ptr) e.pool.emplace(cap, ptr);
}

SpecSet::~SpecSet() {
  if (!dev) return;
  pool_put(*dev, search.buf, search.cap);
  pool_put(*dev, watch.buf, watch.cap);
  pool_put(*dev, gbuf, gcap);
}

// a generator's own device buffers (a borrowed generator's belong to its cache entry)
static void free_gen_buffers(Engine& e, DevGen& g) {
  void free_code(Engine&, DevProgram&);
  if (!g.borrowed) {
    pool_put(e, g.gbuf, g.gcap);
    free_code(e, g.spec);
    free_code(e, g.spec_watch);
  }
  g.gbuf = nullptr;
  free_code(e, g.spec_model);
}

// instructions, literals, lookup lists and coordinate widths in ONE pooled buffer, one copy
static int upload_code(Engine& e, DevProgram& p) {
  p.lds = p.low.value_words <= lds_words_max();
  // MYTHGPU_INTERP_TIERS=0: light or heavy only (the mid variant folded into heavy)
  static const bool tiers = [] {
    const char* g = getenv("MYTHGPU_INTERP_TIERS");
    return !(g && g[0] == '0');
  }();
  p.tier = kTierLight;
  for (const Instr& in : p.low.code) {
    switch (in.op) {
      case K_MUL: case K_SHL: case K_LSHR: case K_ASHR: case K_UMUL_NOOVF:
        p.tier = std::max(p.tier, tiers ? kTierMid : kTierHeavy);
        break;
      case K_UDIV: case K_UREM: case K_SDIV: case K_SREM: case K_SMOD: case K_EXP: p.tier = kTierHeavy; break;
      case K_KECCAK: if (in.a != MG_NONE) p.tier = kTierHeavy; break;
      default: break;
    }
  }
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  // one zeroed Instr past the end: the interpreter prefetches instruction pc + 1
  const size_t b_code = al((p.low.code.size() + 1) * sizeof(Instr)), b_consts = al(p.low.consts.size() * 4),
               b_aux = al(p.low.aux.size() * 4), b_cw = al(p.low.coord_width.size() * 4);
  const size_t total = std::max<size_t>(b_code + b_consts + b_aux + b_cw, 256);
  int rc = pool_get(e, total, &p.buf, &p.cap);
  if (rc) return rc;
  std::vector<uint8_t> h(total, 0);
  std::memcpy(h.data(), p.low.code.data(), p.low.code.size() * sizeof(Instr));
  std::memcpy(h.data() + b_code, p.low.consts.data(), p.low.consts.size() * 4);
  std::memcpy(h.data() + b_code + b_consts, p.low.aux.data(), p.low.aux.size() * 4);
  std::memcpy(h.data() + b_code + b_consts + b_aux, p.low.coord_width.data(), p.low.coord_width.size() * 4);
  HIPCHK(hipMemcpy(p.buf, h.data(), total, hipMemcpyHostToDevice));
  uint8_t* b = (uint8_t*)p.buf;
  p.d_code = (Instr*)b;
  p.d_consts = (uint32_t*)(b + b_code);
  p.d_aux = (uint32_t*)(b + b_code + b_consts);
  p.d_coord_width = (uint32_t*)(b + b_code + b_consts + b_aux);
  p.uploaded = true;
  return MG_OK;
}

void free_code(Engine& e, DevProgram& p) {
  pool_put(e, p.buf, p.cap);
  p.buf = nullptr;
  p.cap = 0;
  p.d_code = nullptr;
  p.d_consts = p.d_aux = p.d_coord_width = nullptr;
  p.uploaded = false;
}

static void fill_info(const DevProgram& p, mg_program_info_t* info) {
  std::memset(info, 0, sizeof(*info));
  info->n_nodes = p.low.n_nodes;
  info->n_instrs = (uint32_t)p.low.code.size();
  info->n_coords = p.low.n_coords;
  info->n_roots = p.low.n_roots;
  info->value_words = p.low.value_words;
  info->uses_lds = p.lds;
  info->n_watch = p.low.n_watch;
  info->watch_words = p.low.watch_words;
  info->coord_words = p.low.coord_words;
  info->limb_ops = p.low.limb_ops;
}

static int ensure_scratch(Engine& e, size_t bytes) {
  if (bytes <= e.scratch_bytes) return MG_OK;
  if (e.d_scratch) (void)hipFree(e.d_scratch);
  e.d_scratch = nullptr;
  e.scratch_bytes = 0;
  HIPCHK(hipMalloc((void**)&e.d_scratch, bytes));
  e.scratch_bytes = bytes;
  return MG_OK;
}

// grid: enough waves to fill 256 CUs several times over, never more than needed.
// Resident waves per CU: the LDS value file (160 KiB per CU) and the VGPRs of the
// kernel variant (heavy ~230: 2 waves/SIMD; mid: 4; light ~50: 8 waves/SIMD).
static uint32_t grid_for(const Engine& e, uint64_t count, bool lds, uint32_t value_words, int tier, int kg = 1,
                         uint32_t extra_bytes = 0) {
  uint64_t want = (count + (uint64_t)kWave * kg - 1) / ((uint64_t)kWave * kg);
  uint32_t waves_per_cu = tier == kTierHeavy ? 8 : tier == kTierMid ? 16 : 32;
  if (lds) {
    const uint32_t bytes = value_words * kWave * 4 * (uint32_t)kg + extra_bytes;
    waves_per_cu = std::max<uint32_t>(1, std::min<uint32_t>(waves_per_cu, (160u * 1024u) / std::max<uint32_t>(bytes, 1)));
  }
  uint64_t cap = (uint64_t)std::max(e.cu_count, 1) * waves_per_cu * 4;
  return (uint32_t)std::max<uint64_t>(1, std::min(want, cap));
}

// k_run's groups per wave per pass: MYTHGPU_INTERP_KG=2|4 where allowed, else 1.  Measured at 2^22
// per launch (profiles/r04n_interp_kg.jsonl): KG 2 / 4 cost C2 35 % / 63 % (5.18 -> 3.35 / 1.94
// G/s), C1 21 % / 53 %, C3 15 % / 44 %, C4 (its file is in global memory: KG 1) unchanged — the
// interpreter waits on LDS and scalar-load latency, which only more resident waves hide, and KG
// divides the waves an LDS-resident value file leaves per CU; the dispatch it amortises is not the
// limiter.  So the default stays 1.
static int interp_kg(int mode, bool lds, bool capture, int tier, uint32_t value_words, uint64_t lanes, int cus) {
  static const int forced = [] {
    const char* g = getenv("MYTHGPU_INTERP_KG");
    const int v = g ? atoi(g) : 0;
    return v == 1 || v == 2 || v == 4 ? v : 0;
  }();
  if (mode == MODE_EVAL || !lds || capture || tier == kTierHeavy) return 1;
  int kg = forced ? forced : 1;
  while (kg > 1 && (value_words * (uint32_t)kg * kWave * 4u > 160u * 1024u ||
                    lanes < (uint64_t)std::max(cus, 1) * 4u * kWave * (uint64_t)kg))
    kg /= 2;
  return kg;
}

// enqueue one interpreter launch on e's stream (e's device must be current); bracketed by
// e.ev0 / e.ev1 so launch_wait can time it
template <int MODE>
static int launch_async(Engine& e, DevProgram& p, KArgs k, uint64_t count) {
  // GEN / SEARCH sweep whole aligned 64-index groups (k_run)
  const uint64_t lanes = MODE == MODE_EVAL ? count : (k.start + count) - (k.start & ~63ull);
  // A launch of at most two waves per CU (a query's first, latency-bound pass) keeps its value file
  // in LDS even past lds_words_max() — up to 64 KiB per one-wave block: the words the global
  // file would fetch from L2 at every operand are what such a launch waits on, and it needs no
  // occupancy.  Larger launches trade the other way (C4 at 255: 20 % slower).
  const bool lds = p.lds || (p.low.value_words <= 255u && lanes <= (uint64_t)std::max(e.cu_count, 1) * 2u * kWave);
  // groups per wave per program pass (k_run KG): one dispatched instruction serves KG x 64 candidates,
  // at KG x the value file in LDS.  Search / gen launches with the file in LDS, no capture, not the
  // heavy tier (its 256-bit temporaries), and a launch big enough to fill the chip at KG
  const int kg = interp_kg(MODE, lds, k.watch != nullptr, p.tier, p.low.value_words, lanes, e.cu_count);
  // MYTHGPU_INTERP_LDS_GEN=1: the prologue copies the generator constants into LDS and dictionary
  // entries are read from there.  Measured slower at 2^22 per launch (profiles/r04z_interp_loadall.jsonl:
  // C2 6.00 -> 5.54 G/s, etherstore 11.1 -> 9.2, C3 23.4 -> 20.5; the copy per block and the smaller
  // occupancy cost more than the L2 gathers), so off by default
  static const bool lds_gen = [] {
    const char* g = getenv("MYTHGPU_INTERP_LDS_GEN");
    return g && g[0] == '1';
  }();
  k.lds_g = kNoLds;
  if (lds && lds_gen && MODE != MODE_EVAL && k.gconsts && k.n_gconsts && k.n_gconsts <= 4096u &&
      (size_t)p.low.value_words * kWave * 4 * kg + (size_t)k.n_gconsts * 4 <= 64u * 1024u)
    k.lds_g = p.low.value_words * kWave * (uint32_t)kg;
  const uint32_t g_bytes = k.lds_g != kNoLds ? k.n_gconsts * 4u : 0u;
  const uint32_t grid = grid_for(e, lanes, lds, p.low.value_words, p.tier, kg, g_bytes);
  k.sk = seed_lane_key(k.seed);
  k.sg = seed_group_key(k.seed);
  k.code = p.d_code;
  k.consts = p.d_consts;
  k.aux = p.d_aux;
  k.coord_width = p.d_coord_width;
  k.count = count;
  k.n_instr = (uint32_t)p.low.code.size();
  k.value_words = p.low.value_words;
  k.n_specs = p.low.n_coords;
  k.pc0 = p.low.n_hoisted;
  // MYTHGPU_INTERP_PREFETCH=0: no scalar-cache warm-up in the prologue
  static const bool prefetch = [] {
    const char* g = getenv("MYTHGPU_INTERP_PREFETCH");
    return !(g && g[0] == '0');
  }();
  if (prefetch) k.flags |= kFlagPrefetch;
  k.stride = (uint64_t)grid * kWave;
  if (!lds) {
    const size_t need = (size_t)p.low.value_words * k.stride * 4;
    int rc = ensure_scratch(e, need);
    if (rc) return rc;
    k.scratch = e.d_scratch;
  }
  const size_t shmem = lds ? (size_t)p.low.value_words * kWave * 4 * kg + g_bytes : 0;
  HIPCHK(hipEventRecord(e.ev0, e.stream));
  const dim3 g(grid), b(kWave);
#define MG_RUN(VFT, TIERC, KGC) hipLaunchKernelGGL((k_run<VFT, MODE, TIERC, KGC>), g, b, shmem, e.stream, k)
  if (lds) {
    if (p.tier == kTierHeavy) {
      MG_RUN(VFLds, kTierHeavy, 1);
    } else if (p.tier == kTierMid) {
      if constexpr (MODE != MODE_EVAL) {
        if (kg == 4) MG_RUN(VFLds, kTierMid, 4);
        else if (kg == 2) MG_RUN(VFLds, kTierMid, 2);
        else MG_RUN(VFLds, kTierMid, 1);
      } else {
        MG_RUN(VFLds, kTierMid, 1);
      }
    } else {
      if constexpr (MODE != MODE_EVAL) {
        if (kg == 4) MG_RUN(VFLds, kTierLight, 4);
        else if (kg == 2) MG_RUN(VFLds, kTierLight, 2);
        else MG_RUN(VFLds, kTierLight, 1);
      } else {
        MG_RUN(VFLds, kTierLight, 1);
      }
    }
  } else {
    if (p.tier == kTierHeavy) MG_RUN(VFGlobal, kTierHeavy, 1);
    else if (p.tier == kTierMid) MG_RUN(VFGlobal, kTierMid, 1);
    else MG_RUN(VFGlobal, kTierLight, 1);
  }
#undef MG_RUN
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e.ev1, e.stream));
  return MG_OK;
}

// wait for e's last launch; its time and `count` candidates go to `st`
static int launch_wait(Engine& e, mg_stats_t& st, uint64_t count) {
  HIPCHK(hipEventSynchronize(e.ev1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e.ev0, e.ev1));
  st.launches++;
  st.last_kernel_ms = ms;
  st.kernel_ms_total += ms;
  st.candidates += count;
  st.last_candidates = count;
  return MG_OK;
}

// reset e's hit buffer before a search launch (async, from pinned memory)
static int arm_hits(Engine& e) {
  // h_hit[0, kHitWords): the armed image (first = ~0, counts 0), written once at init
  HIPCHK(hipMemcpyAsync(e.d_hit, e.h_hit, kHitWords * sizeof(unsigned long long), hipMemcpyHostToDevice, e.stream));
  return MG_OK;
}

// queue the hit buffer's read-back behind e's last launch (async); collect_hits waits for it
static int fetch_hits(Engine& e) {
  HIPCHK(hipMemcpyAsync(e.h_hit + kHitWords, e.d_hit, kHitWords * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        e.stream));
  HIPCHK(hipEventRecord(e.ev2, e.stream));
  return MG_OK;
}

// one wait for launch + read-back; the kernel's time (ev0 -> ev1) and `count` go to `st`
static int collect_hits(Engine& e, mg_stats_t& st, uint64_t count, unsigned long long res[2]) {
  HIPCHK(hipEventSynchronize(e.ev2));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e.ev0, e.ev1));
  st.launches++;
  st.last_kernel_ms = ms;
  st.kernel_ms_total += ms;
  st.candidates += count;
  st.last_candidates = count;
  const unsigned long long* r = e.h_hit + kHitWords;
  res[0] = r[0];
  res[1] = r[1];
  for (uint32_t q = 1; q <= kHitStripes; q++) res[1] += r[kHitStride * q];
  return MG_OK;
}

template <int MODE>
static int launch(Engine& e, DevProgram& p, KArgs k, uint64_t count) {
  if (count == 0) return MG_OK;
  int rc = launch_async<MODE>(e, p, k, count);
  if (rc) return rc;
  return launch_wait(e, e.stats, count);
}

}  // namespace mg

using namespace mg;

extern "C" {

int mg_version(void) { return 2; }

const char* mg_last_error(void) { return g_err.c_str(); }

}  // extern "C"

namespace mg {

// every logical device of the node (mg_init's mask): [0] is E(), the primary, which owns
// the handle tables; the others mirror its programs / generators / JIT kernels under the
// same handles and upload to their device on first use.  Guarded by E().mu.
static std::vector<Engine*> g_devs;

// a search is split over the devices only when every device gets at least this many candidates
// (MYTHGPU_SPLIT_MIN overrides): below it the launch is latency-bound — one launch + one sync on
// device 0, with the model capture, beats N launches + N syncs of a few groups each
static uint64_t split_min_per_device() {
  const char* s = getenv("MYTHGPU_SPLIT_MIN");
  return s ? std::max<uint64_t>(64, strtoull(s, nullptr, 0)) : (uint64_t)1 << 20;
}

static bool split_over_devices(uint64_t count) {
  return g_devs.size() > 1 && count / g_devs.size() >= split_min_per_device();
}

// ---------------------------------------------------------------------------------------------
// The split search's exchange step as ONE RCCL all-reduce(min) over xGMI: after the
// devices' launches are queued, each device's first-hit word (d_hit[0]) is reduced in place on its
// own stream in one ncclGroupStart / ncclGroupEnd, so every device holds the global first hit and
// the host reads it back with the counts.  MYTHGPU_COLLECTIVE=rccl turns it on for a device mask
// that spans distinct physical GPUs (logical devices on one GPU cannot form an RCCL communicator and
// keep the host reduction); =rccl-force also for one device (a one-rank communicator: the plumbing
// on a one-GPU box).  Default: the host reduction (one 2 KiB read per device, which the counts need
// anyway).  librccl is dlopen'ed on first use: no link-time dependency, and a failure to load or to
// build the communicators leaves the host reduction in place (mg_collective_kind says which).
// ---------------------------------------------------------------------------------------------
struct Rccl {
  bool tried = false, ok = false;
  std::string why;
  int (*init_all)(void** comms, int ndev, const int* devlist) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*group_start)() = nullptr;
  int (*group_end)() = nullptr;
  int (*destroy)(void*) = nullptr;
  const char* (*err_str)(int) = nullptr;
  std::vector<void*> comms;  // one per g_devs entry
};
static Rccl g_rccl;
constexpr int kNcclUint64 = 5, kNcclMin = 3;  // rccl.h ncclDataType_t / ncclRedOp_t

static int collective_mode() {  // 0 host, 1 rccl (distinct physical GPUs), 2 rccl-force
  static const int m = [] {
    const char* c = getenv("MYTHGPU_COLLECTIVE");
    if (!c) return 0;
    const std::string v(c);
    return v == "rccl" ? 1 : v == "rccl-force" ? 2 : 0;
  }();
  return m;
}

// caller holds E().mu: the communicators over g_devs, built once; false = host reduction
static bool rccl_ready() {
  Rccl& r = g_rccl;
  if (r.tried) return r.ok;
  r.tried = true;
  const int mode = collective_mode();
  if (!mode) return false;
  std::vector<int> devlist;
  for (Engine* d : g_devs) devlist.push_back(d->device);
  std::vector<int> uniq(devlist);
  std::sort(uniq.begin(), uniq.end());
  if (std::unique(uniq.begin(), uniq.end()) != uniq.end()) {
    r.why = "logical devices share a GPU";
    return false;
  }
  if (devlist.size() < 2 && mode != 2) {
    r.why = "one device";
    return false;
  }
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    r.why = "librccl not found";
    return false;
  }
  r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
  r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
  r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
  r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
  r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
  r.err_str = (decltype(r.err_str))dlsym(h, "ncclGetErrorString");
  if (!r.init_all || !r.all_reduce || !r.group_start || !r.group_end || !r.destroy) {
    r.why = "librccl lacks the symbols";
    return false;
  }
  r.comms.assign(devlist.size(), nullptr);
  const int rc = r.init_all(r.comms.data(), (int)devlist.size(), devlist.data());
  (void)hipSetDevice(E().device);
  if (rc != 0) {
    r.why = std::string("ncclCommInitAll: ") + (r.err_str ? r.err_str(rc) : std::to_string(rc));
    r.comms.clear();
    return false;
  }
  r.ok = true;
  return true;
}

// caller holds E().mu; every device's launch is queued on its stream: d_hit[0] of each device becomes
// the minimum over all of them (in place), ordered before the read-back fetch_hits queues after it
static int rccl_first_hit_min() {
  Rccl& r = g_rccl;
  if (r.group_start() != 0) return set_err(MG_E_HIP, "ncclGroupStart failed");
  int rc = 0;
  for (size_t d = 0; d < g_devs.size() && rc == 0; d++) {
    Engine& de = *g_devs[d];
    rc = r.all_reduce(de.d_hit, de.d_hit, 1, kNcclUint64, kNcclMin, r.comms[d], de.stream);
  }
  const int rc2 = r.group_end();
  (void)hipSetDevice(E().device);
  if (rc != 0 || rc2 != 0)
    return set_err(MG_E_HIP, std::string("ncclAllReduce: ") + (r.err_str ? r.err_str(rc ? rc : rc2) : "error"));
  return MG_OK;
}

static int fetch_hits(Engine& e);

// the split search's exchange (every device takes part: its word is ~0 when it had no slice), then the
// read-back of each device's hit buffer (the counts; word 0 now the global first hit on every device)
static int rccl_fetch(const std::vector<uint64_t>& ct) {
  (void)ct;
  if (int rc = rccl_first_hit_min()) return rc;
  for (Engine* d : g_devs) {
    HIPCHK(hipSetDevice(d->device));
    if (int rc = fetch_hits(*d)) return rc;
  }
  HIPCHK(hipSetDevice(E().device));
  return MG_OK;
}

// One empty launch of every interpreter variant the engine launches by default (and of the capture
// gather and Keccak kernels) at initialisation: the runtime loads a kernel's code on its first launch,
// ~2 ms that the first query of the process paid inside its time to first model (the first k_run
// launch of a process took 1.96 ms against 0.057 ms after, profiles/r04u_cold.jsonl).  An empty
// launch touches no memory: count 0 leaves k_run's group loop empty, rows / n 0 the others.
template <int MODE>
static void warm_run(Engine& e) {
  KArgs k{};
  const dim3 g(1), b(kWave);
  hipLaunchKernelGGL((k_run<VFLds, MODE, kTierLight, 1>), g, b, 0, e.stream, k);
  hipLaunchKernelGGL((k_run<VFLds, MODE, kTierMid, 1>), g, b, 0, e.stream, k);
  hipLaunchKernelGGL((k_run<VFLds, MODE, kTierHeavy, 1>), g, b, 0, e.stream, k);
  hipLaunchKernelGGL((k_run<VFGlobal, MODE, kTierLight, 1>), g, b, 0, e.stream, k);
  hipLaunchKernelGGL((k_run<VFGlobal, MODE, kTierMid, 1>), g, b, 0, e.stream, k);
  hipLaunchKernelGGL((k_run<VFGlobal, MODE, kTierHeavy, 1>), g, b, 0, e.stream, k);
}

static int warm_kernels(Engine& e) {
  static const bool off = [] {
    const char* g = getenv("MYTHGPU_WARM_KERNELS");
    return g && g[0] == '0';
  }();
  if (off) return MG_OK;
  warm_run<MODE_EVAL>(e);
  warm_run<MODE_GEN>(e);
  warm_run<MODE_SEARCH>(e);
  hipLaunchKernelGGL(k_gather_rows, dim3(1), dim3(256), 0, e.stream, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u);
  hipLaunchKernelGGL(k_keccak, dim3(1), dim3(256), 0, e.stream, (const uint8_t*)nullptr, (const uint64_t*)nullptr,
                     (const uint32_t*)nullptr, (uint64_t)0, (uint8_t*)nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(e.stream));
  return MG_OK;
}

static int init_dev(Engine& e, int dev) {
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, dev));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    return set_err(MG_E_NODEVICE, std::string("device is ") + prop.gcnArchName + ", engine is built for gfx950");
  HIPCHK(hipSetDevice(dev));
  // the host waits on every search result: spin instead of sleeping on an interrupt (a
  // no-op when the device's context already exists, e.g. torch created it first)
  (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
  HIPCHK(hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreate(&e.ev0));
  HIPCHK(hipEventCreate(&e.ev1));
  HIPCHK(hipEventCreateWithFlags(&e.ev2, hipEventDisableTiming));
  HIPCHK(hipMalloc((void**)&e.d_hit, kHitAlloc * sizeof(unsigned long long)));
  HIPCHK(hipMemset(e.d_hit + kPeerWord, 0, (1 + kPeerMax) * sizeof(unsigned long long)));  // no peers
  HIPCHK(hipHostMalloc((void**)&e.h_hit, 2 * kHitWords * sizeof(unsigned long long), hipHostMallocDefault));
  std::memset(e.h_hit, 0, 2 * kHitWords * sizeof(unsigned long long));
  e.h_hit[0] = ~0ull;  // the armed image (arm_hits)
  // the model-capture buffer of latency-bound searches (mg_search), allocated up front so that no
  // query's time to first model includes the allocation
  HIPCHK(hipMalloc((void**)&e.d_capture, kCaptureBytes));
  e.capture_bytes = kCaptureBytes;
  e.device = dev;
  e.cu_count = prop.multiProcessorCount;
  e.clock_mhz = prop.clockRate / 1000;
  e.stats.device = dev;
  e.stats.cu_count = e.cu_count;
  e.stats.clock_mhz = e.clock_mhz;
  e.init = true;
  return warm_kernels(e);
}

static void free_dev_buffers(Engine& e);

}  // namespace mg

extern "C" {

int mg_init(uint32_t device_mask) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  if (e.init) return MG_OK;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return set_err(MG_E_NODEVICE, "no HIP device");
  std::vector<int> devs;
  for (int d = 0; d < n && d < 32; d++)
    if (device_mask & (1u << d)) devs.push_back(d);
  if (devs.empty()) devs.push_back(0);
  // MYTHGPU_VIRTUAL_DEVICES=k: k logical devices on the first physical one (own streams and
  // buffers) — exercises the multi-device split and reduction on a one-GPU machine
  if (const char* v = getenv("MYTHGPU_VIRTUAL_DEVICES")) {
    const int k = std::max(1, std::min(16, atoi(v)));
    devs.assign((size_t)k, devs[0]);
  }
  int rc = init_dev(e, devs[0]);
  if (rc) return rc;
  g_devs.assign(1, &e);
  for (size_t i = 1; i < devs.size(); i++) {
    Engine* s2 = new Engine;  // freed by mg_shutdown
    rc = init_dev(*s2, devs[i]);
    if (rc) {
      // all or nothing: a retry must not run on fewer devices than the mask asked for
      const std::string why = g_err;
      if (s2->init) free_dev_buffers(*s2);
      delete s2;
      for (size_t k = g_devs.size(); k-- > 0;) {
        (void)hipSetDevice(g_devs[k]->device);
        free_dev_buffers(*g_devs[k]);
        if (g_devs[k] != &e) delete g_devs[k];
      }
      g_devs.clear();
      e.init = false;
      return set_err(rc, "mg_init: device " + std::to_string(devs[i]) + ": " + why);
    }
    g_devs.push_back(s2);
  }
  // peer lines: device d stops devices d+1.. (their slices lie above its own).  Distinct physical
  // devices need peer access (xGMI); where it cannot be enabled, that pair simply does not stop early
  if (g_devs.size() > 1) {
    // Memory model of the stop words.  Each device's first-hit word is lowered by its own waves
    // (agent-scope atomics) and by waves of the devices below it (the peer line).  When those are
    // other GPUs, their atomics cross xGMI: the hit buffers are then allocated fine-grained
    // (hipDeviceMallocFinegrained), peers publish with system-scope atomics (publish_peers; the
    // kernels' sc1 atomics) which the owner's memory performs, and the owner's waves read the word
    // with system-scope loads (MG_SEARCH_SYSTEM_SCOPE: sc0 sc1, which no cache level serves stale).
    // Virtual devices on one GPU (MYTHGPU_VIRTUAL_DEVICES) keep coarse-grained buffers and agent
    // scope.  A late or lost peer write costs only the early stop: the host takes the minimum over
    // every device's word.
    bool physical = false;
    for (size_t d = 1; d < g_devs.size(); d++) physical = physical || g_devs[d]->device != g_devs[0]->device;
    if (physical) {
      for (Engine* de : g_devs) {
        HIPCHK(hipSetDevice(de->device));
        HIPCHK(hipFree(de->d_hit));
        de->d_hit = nullptr;
        HIPCHK(hipExtMallocWithFlags((void**)&de->d_hit, kHitAlloc * sizeof(unsigned long long), hipDeviceMallocFinegrained));
        HIPCHK(hipMemset(de->d_hit, 0, kHitAlloc * sizeof(unsigned long long)));
        de->sys_scope = true;
      }
    }
    for (size_t d = 0; d < g_devs.size(); d++) {
      std::vector<unsigned long long> line(1 + kPeerMax, 0ull);
      uint32_t np = 0;
      for (size_t q = d + 1; q < g_devs.size() && np < kPeerMax; q++) {
        const int a = g_devs[d]->device, b = g_devs[q]->device;
        if (a != b) {
          int can = 0;
          if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
          (void)hipSetDevice(a);
          const hipError_t pe = hipDeviceEnablePeerAccess(b, 0);
          if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
            (void)hipGetLastError();
            continue;
          }
        }
        line[1 + np++] = (unsigned long long)(uintptr_t)g_devs[q]->d_hit;
      }
      line[0] = np;
      HIPCHK(hipSetDevice(g_devs[d]->device));
      HIPCHK(hipMemcpy(g_devs[d]->d_hit + kPeerWord, line.data(), line.size() * sizeof(unsigned long long),
                       hipMemcpyHostToDevice));
    }
  }
  HIPCHK(hipSetDevice(e.device));
  e.stats.n_devices = (uint32_t)g_devs.size();
  {
    std::lock_guard<std::mutex> wl(g_warm_mu);
    g_warm_running++;
  }
  std::thread([] {  // helpers up (and the first tier's assembler warm) before the first query needs them
    struct Done {  // mg_shutdown / the exit handler wait for this before stopping the helpers
      ~Done() {
        std::lock_guard<std::mutex> wl(g_warm_mu);
        g_warm_running--;
        g_warm_cv.notify_all();
      }
    } done_;
    Lowered P;
    P.vwidth = {1};
    P.consts = {1};
    P.vcode = {Instr{K_CONST, 1, 0, MG_NONE, MG_NONE, MG_NONE, 0, 0},
               Instr{K_ASSERT, 1, MG_NONE, 0, MG_NONE, MG_NONE, 0, 0}};
    std::string src, err;
    if (jit_asm_source(P, {}, {}, JIT_EVAL, src, err) != MG_OK) src.clear();
    jit_helper_warm(src);
  }).detach();
  return MG_OK;
}

int mg_split_range(uint64_t start, uint64_t count, uint32_t n_dev, uint64_t* starts, uint64_t* counts) {
  if (n_dev == 0 || !starts || !counts) return set_err(MG_E_INVALID, "mg_split_range: bad arguments");
  // whole aligned 64-index groups per device (one group = one wave, GEN3 group key), in
  // index order: device d scans the d-th contiguous slice
  const uint64_t end = start + count, a0 = start & ~63ull;
  const uint64_t ngroups = count ? (end - a0 + 63ull) >> 6 : 0;
  for (uint32_t d = 0; d < n_dev; d++) {
    const uint64_t g0 = ngroups * d / n_dev, g1 = ngroups * (d + 1) / n_dev;
    const uint64_t lo = std::max<uint64_t>(start, a0 + 64ull * g0), hi = std::min<uint64_t>(end, a0 + 64ull * g1);
    starts[d] = lo;
    counts[d] = hi > lo ? hi - lo : 0;
  }
  return MG_OK;
}

void mg_shutdown(void) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  {
    // stop the compile thread (a compile in flight finishes first; its result is dropped)
    std::unique_lock<std::mutex> jl(e.jit_mu);
    e.jit_stop = true;
    for (auto& q : e.jit_queue)
      for (auto& t : q) t->cancelled = true;
    for (auto& kv : e.tickets) kv.second->cancelled = true;
    e.jit_cv.notify_all();
    e.jit_done_cv.wait(jl, [&] { return e.jit_workers == 0; });
    e.jit_stop = false;
    for (auto& q : e.jit_queue) q.clear();
    for (auto& kv : e.tickets)
      if (kv.second->ready) release_jit(*kv.second->ready);
    e.tickets.clear();
  }
  wait_warm();        // the warm-up's helper requests end before the helpers stop
  jit_helper_stop();  // the compiler process ends on end of input (started again on demand)
  if (!e.init) {
    for (auto& kv : e.jits) release_jit(*kv.second);
    e.jits.clear();
    e.code_cache.lru.clear();
    e.code_cache.idx.clear();
    return;
  }
  if (g_rccl.ok) {  // the communicators before the streams and buffers they use
    for (void* c : g_rccl.comms) (void)g_rccl.destroy(c);
    g_rccl.comms.clear();
  }
  g_rccl.tried = g_rccl.ok = false;
  for (size_t i = g_devs.size(); i-- > 0;) {
    Engine* d = g_devs[i];
    (void)hipSetDevice(d->device);
    free_dev_buffers(*d);
    if (d != &e) delete d;
  }
  g_devs.clear();
}

}  // extern "C"

namespace mg {

// every device buffer, module and stream of one logical device (its device current)
static void free_dev_buffers(Engine& e) {
  for (auto& kv : e.jits) release_jit(*kv.second);
  e.jits.clear();
  e.code_cache.lru.clear();  // the resident modules
  e.code_cache.idx.clear();
  for (auto& kv : e.progs) free_code(e, *kv.second);
  e.progs.clear();
  for (auto& kv : e.gens) free_gen_buffers(e, *kv.second);
  e.gens.clear();
  // the cache's resident specialisations return their buffers to the pool before it is freed
  e.spec_cache.clear();
  e.spec_order.clear();
  for (auto& kv : e.pool) (void)hipFree(kv.second);
  e.pool.clear();
  if (e.d_watch1) (void)hipFree(e.d_watch1);
  if (e.d_ver1) (void)hipFree(e.d_ver1);
  e.d_watch1 = nullptr;
  e.d_ver1 = nullptr;
  e.watch1_words = 0;
  if (e.d_capture) (void)hipFree(e.d_capture);
  e.d_capture = nullptr;
  e.capture_bytes = 0;
  if (e.d_scratch) (void)hipFree(e.d_scratch);
  e.d_scratch = nullptr;
  e.scratch_bytes = 0;
  (void)hipFree(e.d_hit);
  if (e.h_hit) (void)hipHostFree(e.h_hit);
  if (e.d_hitmany) (void)hipFree(e.d_hitmany);
  if (e.h_hitmany) (void)hipHostFree(e.h_hitmany);
  e.d_hitmany = nullptr;
  e.h_hitmany = nullptr;
  for (int q = 0; q < 4; q++) {
    if (e.xs[q]) (void)hipStreamDestroy(e.xs[q]);
    if (e.xev[q]) (void)hipEventDestroy(e.xev[q]);
    e.xs[q] = nullptr;
    e.xev[q] = nullptr;
  }
  if (e.h_watch1) (void)hipHostFree(e.h_watch1);
  e.h_hit = nullptr;
  e.h_watch1 = nullptr;
  e.h_watch1_words = 0;
  (void)hipEventDestroy(e.ev0);
  (void)hipEventDestroy(e.ev1);
  (void)hipEventDestroy(e.ev2);
  (void)hipStreamDestroy(e.stream);
  e.init = false;
}

}  // namespace mg

extern "C" {

int mg_program_check(const uint8_t* ssa, size_t len, mg_program_info_t* info) {
  Lowered low;
  std::string err;
  int rc = lower_program(ssa, len, low, err);
  if (rc) return set_err(rc, err);
  if (info) {
    std::memset(info, 0, sizeof(*info));
    info->n_nodes = low.n_nodes;
    info->n_instrs = (uint32_t)low.code.size();
    info->n_coords = low.n_coords;
    info->n_roots = low.n_roots;
    info->value_words = low.value_words;
    info->uses_lds = low.value_words <= lds_words_max();
    info->n_watch = low.n_watch;
    info->watch_words = low.watch_words;
    info->coord_words = low.coord_words;
    info->limb_ops = low.limb_ops;
  }
  return MG_OK;
}

int mg_program_check_gen(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words,
                         mg_program_info_t* info) {
  DevProgram base, sp;
  std::string err;
  int rc = lower_program(ssa, len, base.low, err);
  if (rc) return set_err(rc, err);
  std::vector<GenSpec> specs;
  std::vector<uint32_t> consts;
  rc = parse_gen(base.low, gen_blob, gen_words, specs, consts, err);
  if (rc) return set_err(rc, err);
  rc = specialize_program(base.low, &specs, &consts, sp.low, err);
  if (rc) return set_err(rc, err);
  sp.lds = sp.low.value_words <= lds_words_max();
  if (info) fill_info(sp, info);
  return MG_OK;
}

int mg_program_specialized(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words,
                           uint32_t flags, uint32_t* buf, size_t cap_words, size_t* out_words) {
  Lowered base, sp;
  std::string err;
  int rc = lower_program(ssa, len, base, err);
  if (rc) return set_err(rc, err);
  std::vector<GenSpec> specs;
  std::vector<uint32_t> consts;
  if (gen_blob) {
    rc = parse_gen(base, gen_blob, gen_words, specs, consts, err);
    if (rc) return set_err(rc, err);
  }
  rc = specialize_program(base, gen_blob ? &specs : nullptr, gen_blob ? &consts : nullptr, sp, err,
                          (flags & MG_SPEC_KEEP_WATCH) != 0);
  if (rc) return set_err(rc, err);
  // MG_SPEC_INTERP: the interpreter's program where it differs from the JIT's
  const bool interp = (flags & MG_SPEC_INTERP) && !sp.ivcode.empty();
  const std::vector<Instr>& code = interp ? sp.ivcode : sp.vcode;
  const std::vector<uint32_t>& aux = interp ? sp.ivaux : sp.vaux;
  std::vector<uint32_t> w = {MG_SPEC_MAGIC, (uint32_t)code.size(), (uint32_t)sp.consts.size(),
                             (uint32_t)aux.size(), (uint32_t)sp.vwidth.size(), sp.n_coords};
  for (const Instr& in : code) w.insert(w.end(), &in.op, &in.op + 8);
  w.insert(w.end(), sp.consts.begin(), sp.consts.end());
  w.insert(w.end(), aux.begin(), aux.end());
  w.insert(w.end(), sp.vwidth.begin(), sp.vwidth.end());
  if (out_words) *out_words = w.size();
  if (buf == nullptr || cap_words < w.size()) return buf == nullptr ? MG_OK : set_err(MG_E_INVALID, "buffer too small");
  std::memcpy(buf, w.data(), 4 * w.size());
  return MG_OK;
}

int mg_program_load(const uint8_t* ssa, size_t len, uint64_t* handle) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  if (!e.init) return set_err(MG_E_NOTINIT, "mg_init not called");
  auto p = std::make_unique<DevProgram>();
  p->src.assign((const char*)ssa, len);
  auto hit = e.lower_cache.find(p->src);
  if (hit != e.lower_cache.end()) {
    p->low = *hit->second;
  } else {
    std::string err;
    int rc = lower_program(ssa, len, p->low, err);
    if (rc) return set_err(rc, err);
    e.lower_cache[p->src] = std::make_shared<Lowered>(p->low);
    e.lower_order.push_back(p->src);
    if (e.lower_order.size() > e.cache_cap) {
      e.lower_cache.erase(e.lower_order.front());
      e.lower_order.pop_front();
    }
  }
  // uploaded on first use: searches run the generator-specialised copies (mg_gen_load),
  // only explicit-coordinate evaluation runs this one
  const uint64_t h = e.next_handle++;
  for (size_t i = 1; i < g_devs.size(); i++) {  // the other devices: same handle, uploaded on use
    auto q = std::make_unique<DevProgram>();
    q->low = p->low;
    g_devs[i]->progs[h] = std::move(q);
  }
  e.progs[h] = std::move(p);
  e.stats.programs_loaded++;
  *handle = h;
  return MG_OK;
}

static DevProgram* find_prog(Engine& e, uint64_t h) {
  auto it = e.progs.find(h);
  return it == e.progs.end() ? nullptr : it->second.get();
}

int mg_program_info(uint64_t prog, mg_program_info_t* info) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  DevProgram* p = find_prog(e, prog);
  if (!p) return set_err(MG_E_INVALID, "bad program handle");
  fill_info(*p, info);
  return MG_OK;
}

int mg_gen_info(uint64_t gen, mg_program_info_t* info) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.gens.find(gen);
  if (it == e.gens.end()) return set_err(MG_E_INVALID, "bad generator handle");
  fill_info(it->second->spec, info);
  return MG_OK;
}

int mg_program_free(uint64_t prog) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.progs.find(prog);
  if (it == e.progs.end()) return set_err(MG_E_INVALID, "bad program handle");
  free_code(e, *it->second);
  e.progs.erase(it);
  for (size_t i = 1; i < g_devs.size(); i++) {
    Engine& d = *g_devs[i];
    auto q = d.progs.find(prog);
    if (q == d.progs.end()) continue;
    free_code(d, *q->second);  // pooled on that device (no device call)
    d.progs.erase(q);
  }
  return MG_OK;
}

}  // extern "C"

namespace mg {

// specs | consts in one pooled buffer on e's device (current)
static int upload_gen_consts(Engine& e, DevGen& gg) {
  const size_t b_specs = (gg.specs.size() * sizeof(GenSpec) + 255) & ~(size_t)255;
  const size_t total = std::max<size_t>(b_specs + gg.consts.size() * 4, 256);
  int rc = pool_get(e, total, &gg.gbuf, &gg.gcap);
  if (rc) return rc;
  std::vector<uint8_t> h(total, 0);
  std::memcpy(h.data(), gg.specs.data(), gg.specs.size() * sizeof(GenSpec));
  std::memcpy(h.data() + b_specs, gg.consts.data(), gg.consts.size() * 4);
  HIPCHK(hipMemcpy(gg.gbuf, h.data(), total, hipMemcpyHostToDevice));
  gg.d_specs = (GenSpec*)gg.gbuf;
  gg.d_consts = (uint32_t*)((uint8_t*)gg.gbuf + b_specs);
  return MG_OK;
}

// a mirrored generator's search program + constants on device d (d's device current)
static int ensure_gen_on(Engine& d, DevGen& gg) {
  int rc;
  if (!gg.spec.uploaded && (rc = upload_code(d, gg.spec))) return rc;
  if (!gg.gbuf && (rc = upload_gen_consts(d, gg))) return rc;
  return MG_OK;
}

}  // namespace mg

extern "C" {

int mg_gen_load(uint64_t prog, const uint32_t* blob, size_t n_words, uint64_t* gen_handle) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  DevProgram* p = find_prog(e, prog);
  if (!p) return set_err(MG_E_INVALID, "bad program handle");
  std::vector<GenSpec> specs;
  std::vector<uint32_t> consts;
  std::string err;
  int rc = parse_gen(p->low, blob, n_words, specs, consts, err);
  if (rc) return set_err(rc, err);
  auto gg = std::make_unique<DevGen>();
  gg->prog = prog;
  gg->specs = specs;
  gg->consts = consts;
  const std::string key = p->src + std::string((const char*)blob, n_words * 4);
  std::shared_ptr<SpecSet> sp;
  auto hit = e.spec_cache.find(key);
  if (hit != e.spec_cache.end()) {
    sp = hit->second;
  } else {
    sp = std::make_shared<SpecSet>();
    rc = specialize_program(p->low, &gg->specs, &gg->consts, sp->search.low, err, /*keep_watch=*/false);
    if (rc) return set_err(rc, err);
    rc = specialize_program(p->low, &gg->specs, &gg->consts, sp->watch.low, err, /*keep_watch=*/true);
    if (rc) return set_err(rc, err);
  }
  if (!sp->dev) {  // upload once: code of both variants, then specs | constants
    if ((rc = upload_code(e, sp->search))) return rc;
    if ((rc = upload_code(e, sp->watch))) return rc;
    if ((rc = upload_gen_consts(e, *gg))) return rc;
    sp->gbuf = gg->gbuf;
    sp->gcap = gg->gcap;
    sp->d_specs = gg->d_specs;
    sp->d_consts = gg->d_consts;
    sp->dev = &e;
  }
  if (hit == e.spec_cache.end()) {
    e.spec_cache[key] = sp;
    e.spec_order.push_back(key);
    if (e.spec_order.size() > e.cache_cap) {
      e.spec_cache.erase(e.spec_order.front());
      e.spec_order.pop_front();
    }
  }
  gg->set = sp;
  gg->spec = sp->search;
  gg->spec_watch = sp->watch;
  gg->gbuf = nullptr;
  gg->gcap = 0;
  gg->d_specs = sp->d_specs;
  gg->d_consts = sp->d_consts;
  gg->borrowed = true;
  const uint64_t h = e.next_handle++;
  for (size_t i = 1; i < g_devs.size(); i++) {  // mirrored, uploaded on first use there
    auto q = std::make_unique<DevGen>();
    q->prog = prog;
    q->specs = gg->specs;
    q->consts = gg->consts;
    q->spec.low = gg->spec.low;
    q->spec_watch.low = gg->spec_watch.low;
    g_devs[i]->gens[h] = std::move(q);
  }
  e.gens[h] = std::move(gg);
  *gen_handle = h;
  return MG_OK;
}

int mg_gen_free(uint64_t gen) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.gens.find(gen);
  if (it == e.gens.end()) return set_err(MG_E_INVALID, "bad generator handle");
  for (size_t i = 0; i < g_devs.size(); i++) {
    Engine& d = *g_devs[i];
    auto q = d.gens.find(gen);
    if (q == d.gens.end()) continue;
    free_gen_buffers(d, *q->second);
    d.gens.erase(q);
  }
  if (g_devs.empty()) {
    free_gen_buffers(e, *it->second);
    e.gens.erase(it);
  }
  return MG_OK;
}

int mg_eval_dev(uint64_t prog, const uint32_t* d_soa, uint64_t n, uint8_t* d_verdict, uint32_t* d_watch) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  DevProgram* p = find_prog(e, prog);
  if (!p) return set_err(MG_E_INVALID, "bad program handle");
  if (!p->uploaded) {
    int rc = upload_code(e, *p);
    if (rc) return rc;
  }
  KArgs k{};
  k.soa = d_soa;
  k.verdict = d_verdict;
  k.watch = d_watch;
  k.start = 0;
  return launch<MODE_EVAL>(e, *p, k, n);
}

int mg_eval(uint64_t prog, const uint32_t* soa, uint64_t n, uint8_t* verdict_out, uint32_t* watch_out) {
  Engine& e = E();
  DevProgram* p;
  {
    std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
    if (!e.init) return set_err(MG_E_NOTINIT, "mg_init not called");
    p = find_prog(e, prog);
    if (!p) return set_err(MG_E_INVALID, "bad program handle");
  }
  if (n == 0) return MG_OK;
  const size_t soa_bytes = (size_t)std::max<uint32_t>(p->low.coord_words, 1) * n * 4;
  const size_t watch_bytes = (size_t)p->low.watch_words * n * 4;
  uint32_t *d_soa = nullptr, *d_watch = nullptr;
  uint8_t* d_ver = nullptr;
  HIPCHK(hipMalloc((void**)&d_soa, soa_bytes));
  HIPCHK(hipMalloc((void**)&d_ver, n));
  if (watch_out && watch_bytes) HIPCHK(hipMalloc((void**)&d_watch, watch_bytes));
  if (p->low.coord_words) HIPCHK(hipMemcpy(d_soa, soa, (size_t)p->low.coord_words * n * 4, hipMemcpyHostToDevice));
  int rc = mg_eval_dev(prog, d_soa, n, d_ver, d_watch);
  if (rc == MG_OK) {
    HIPCHK(hipMemcpy(verdict_out, d_ver, n, hipMemcpyDeviceToHost));
    if (d_watch) HIPCHK(hipMemcpy(watch_out, d_watch, watch_bytes, hipMemcpyDeviceToHost));
  }
  (void)hipFree(d_soa);
  (void)hipFree(d_ver);
  if (d_watch) (void)hipFree(d_watch);
  return rc;
}

int mg_eval_generated(uint64_t prog, uint64_t gen, uint64_t seed, uint64_t start, uint64_t n, uint8_t* verdict_out,
                      uint32_t* watch_out) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  DevProgram* p = find_prog(e, prog);
  if (!p) return set_err(MG_E_INVALID, "bad program handle");
  auto it = e.gens.find(gen);
  if (it == e.gens.end() || it->second->prog != prog) return set_err(MG_E_INVALID, "bad generator handle");
  if (n == 0) return MG_OK;
  const size_t watch_bytes = (size_t)p->low.watch_words * n * 4;
  uint32_t* d_watch = nullptr;
  uint8_t* d_ver = nullptr;
  HIPCHK(hipMalloc((void**)&d_ver, n));
  if (watch_out && watch_bytes) HIPCHK(hipMalloc((void**)&d_watch, watch_bytes));
  KArgs k{};
  k.specs = it->second->d_specs;
  k.gconsts = it->second->d_consts;
  k.n_gconsts = (uint32_t)it->second->consts.size();
  k.verdict = d_ver;
  k.watch = d_watch;
  k.start = start;
  k.seed = seed;
  int rc = launch<MODE_GEN>(e, it->second->spec_watch, k, n);
  if (rc == MG_OK) {
    HIPCHK(hipMemcpy(verdict_out, d_ver, n, hipMemcpyDeviceToHost));
    if (d_watch) HIPCHK(hipMemcpy(watch_out, d_watch, watch_bytes, hipMemcpyDeviceToHost));
  }
  (void)hipFree(d_ver);
  if (d_watch) (void)hipFree(d_watch);
  return rc;
}

// the model of candidate `idx`: the watch rows of the generator's watch-list variant
// (one interpreter lane; ~tens of microseconds) -> assign_out[watch_words]
static int read_assignment(Engine& e, DevGen& g, uint64_t seed, uint64_t idx, uint32_t* assign_out) {
  const uint32_t ww = g.spec_watch.low.watch_words;
  if (ww == 0) return MG_OK;
  // the model of a known hit: the watch list's slice of the program only (no asserts), a
  // shorter single-candidate pass than the full keep_watch program
  if (!g.spec_model.uploaded) {
    if (!g.set || !g.set->model) {
      DevProgram* p = find_prog(e, g.prog);
      if (!p) return set_err(MG_E_INVALID, "bad program handle");
      auto m = std::make_shared<Lowered>();
      std::string err;
      int rc = specialize_program(p->low, &g.specs, &g.consts, *m, err, /*keep_watch=*/true, /*keep_asserts=*/false);
      if (rc) return set_err(rc, err);
      if (!g.set) g.set = std::make_shared<SpecSet>();
      g.set->model = m;
    }
    g.spec_model.low = *g.set->model;
    int rc = upload_code(e, g.spec_model);
    if (rc) return rc;
  }
  if (g.spec_model.low.watch_words != ww) return set_err(MG_E_INVALID, "internal: model read-back layout");
  if (ww > e.watch1_words) {
    if (e.d_watch1) (void)hipFree(e.d_watch1);
    e.d_watch1 = nullptr;
    e.watch1_words = 0;
    HIPCHK(hipMalloc((void**)&e.d_watch1, (size_t)ww * 4));
    e.watch1_words = ww;
  }
  if (!e.d_ver1) HIPCHK(hipMalloc((void**)&e.d_ver1, 64));
  KArgs k{};
  k.specs = g.d_specs;
  k.gconsts = g.d_consts;
  k.n_gconsts = (uint32_t)g.consts.size();
  k.verdict = e.d_ver1;
  k.watch = e.d_watch1;
  k.start = idx;
  k.seed = seed;
  if (ww > e.h_watch1_words) {
    if (e.h_watch1) (void)hipHostFree(e.h_watch1);
    e.h_watch1 = nullptr;
    e.h_watch1_words = 0;
    HIPCHK(hipHostMalloc((void**)&e.h_watch1, (size_t)ww * 4, hipHostMallocDefault));
    e.h_watch1_words = ww;
  }
  int rc = launch_async<MODE_GEN>(e, g.spec_model, k, 1);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(e.h_watch1, e.d_watch1, (size_t)ww * 4, hipMemcpyDeviceToHost, e.stream));
  HIPCHK(hipEventRecord(e.ev2, e.stream));
  HIPCHK(hipEventSynchronize(e.ev2));
  std::memcpy(assign_out, e.h_watch1, (size_t)ww * 4);
  return MG_OK;
}

int mg_search(uint64_t prog, uint64_t gen, uint64_t seed, uint64_t start, uint64_t count, uint32_t flags,
              uint64_t* first_hit, uint64_t* n_hits, uint32_t* assign_out) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  DevProgram* p = find_prog(e, prog);
  if (!p) return set_err(MG_E_INVALID, "bad program handle");
  auto it = e.gens.find(gen);
  if (it == e.gens.end() || it->second->prog != prog) return set_err(MG_E_INVALID, "bad generator handle");
  unsigned long long res[2] = {~0ull, 0ull};
  if (split_over_devices(count)) {
    // the node's devices each sweep one contiguous, group-aligned slice (mg_split_range) on
    // their own stream; first hit = min, hits = sum over the slices (a host reduction: one
    // 16-byte read per device, no collective needed inside one process)
    const uint32_t nd = (uint32_t)g_devs.size();
    std::vector<uint64_t> st(nd), ct(nd);
    mg_split_range(start, count, nd, st.data(), ct.data());
    int rc = MG_OK;
    const bool coll = rccl_ready();  // the exchange as one RCCL all-reduce(min) (MYTHGPU_COLLECTIVE)
    for (uint32_t d = 0; d < nd && rc == MG_OK; d++) {
      if (!ct[d]) continue;
      Engine& de = *g_devs[d];
      HIPCHK(hipSetDevice(de.device));
      DevGen& dg = *de.gens.at(gen);
      if ((rc = ensure_gen_on(de, dg))) break;
      if ((rc = arm_hits(de))) break;
      KArgs k{};
      k.specs = dg.d_specs;
      k.gconsts = dg.d_consts;
      k.n_gconsts = (uint32_t)dg.consts.size();
      k.first_hit = de.d_hit;
      k.hits = de.d_hit + 1;
      k.start = st[d];
      k.seed = seed;
      k.flags = flags | (de.sys_scope ? MG_SEARCH_SYSTEM_SCOPE : 0u);
      rc = launch_async<MODE_SEARCH>(de, dg.spec, k, ct[d]);
      if (rc == MG_OK && !coll) rc = fetch_hits(de);
    }
    if (rc == MG_OK && coll) rc = rccl_fetch(ct);
    for (uint32_t d = 0; d < nd; d++) {
      if (!ct[d]) continue;
      Engine& de = *g_devs[d];
      (void)hipSetDevice(de.device);
      unsigned long long r[2];
      if (rc == MG_OK) rc = collect_hits(de, e.stats, ct[d], r);
      if (rc == MG_OK) {
        res[0] = std::min(res[0], r[0]);
        res[1] += r[1];
      }
    }
    HIPCHK(hipSetDevice(e.device));
    if (rc) return rc;
  } else {
    KArgs k{};
    k.specs = it->second->d_specs;
    k.gconsts = it->second->d_consts;
    k.n_gconsts = (uint32_t)it->second->consts.size();
    k.first_hit = e.d_hit;
    k.hits = e.d_hit + 1;
    k.start = start;
    k.seed = seed;
    k.flags = flags;
    if (count) {
      DevGen& dg = *it->second;
      const uint32_t ww = dg.spec_watch.low.watch_words;
      const uint64_t lanes = (start + count) - (start & ~63ull);
      // a latency-bound launch (every block sweeps one 64-index group, e.g. the first launch of
      // a get_model query) runs the program with its watch list and captures every lane's
      // watch rows, so a hit's model needs no second pass (read_assignment); the capture buffer
      // is blocks x watch_words x 64 words
      const DevProgram& pw = dg.spec_watch;
      const uint32_t grid_w = grid_for(e, lanes, pw.lds, pw.low.value_words, pw.tier);
      const bool capture = assign_out && ww && pw.uploaded && lanes <= (uint64_t)grid_w * kWave &&
                           (uint64_t)grid_w * ww * kWave * 4u <= kCaptureBytes;
      int rc = MG_OK;
      if (capture) {
        // allocated once per device (64 MiB) and the staging rows pinned, so a query's first
        // search pays neither an allocation nor a pageable copy
        if (!e.d_capture) {
          HIPCHK(hipMalloc((void**)&e.d_capture, kCaptureBytes));
          e.capture_bytes = kCaptureBytes;
        }
        if (ww > e.h_watch1_words) {
          if (e.h_watch1) (void)hipHostFree(e.h_watch1);
          e.h_watch1 = nullptr;
          e.h_watch1_words = 0;
          HIPCHK(hipHostMalloc((void**)&e.h_watch1, (size_t)ww * 4, hipHostMallocDefault));
          e.h_watch1_words = ww;
        }
        k.watch = e.d_capture;
        k.watch_words = ww;
      }
      rc = arm_hits(e);
      if (!rc) rc = launch_async<MODE_SEARCH>(e, capture ? dg.spec_watch : dg.spec, k, count);
      if (!rc) rc = fetch_hits(e);
      if (!rc) rc = collect_hits(e, e.stats, count, res);
      if (rc) return rc;
      if (capture) {
        if (first_hit) *first_hit = res[0];
        if (n_hits) *n_hits = res[1];
        e.stats.hits += res[1];
        if (res[0] == ~0ull) return MG_OK;
        // the hit's block (one group per block, in order) and lane
        const uint64_t off = res[0] - (start & ~63ull);
        const uint64_t b = off / kWave, lane = off % kWave;
        // gather the lane's column on the device (a 2-D copy would load HIP's blit kernel on
        // first use, milliseconds inside a cold query), then one contiguous read-back
        if (ww > e.watch1_words) {
          if (e.d_watch1) (void)hipFree(e.d_watch1);
          e.d_watch1 = nullptr;
          e.watch1_words = 0;
          HIPCHK(hipMalloc((void**)&e.d_watch1, (size_t)ww * 4));
          e.watch1_words = ww;
        }
        const uint32_t* src = e.d_capture + (b * ww) * kWave + lane;
        hipLaunchKernelGGL(k_gather_rows, dim3((ww + 255) / 256), dim3(256), 0, e.stream, src, e.d_watch1, ww);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(e.h_watch1, e.d_watch1, (size_t)ww * 4, hipMemcpyDeviceToHost, e.stream));
        HIPCHK(hipStreamSynchronize(e.stream));
        std::memcpy(assign_out, e.h_watch1, (size_t)ww * 4);
        return MG_OK;
      }
    }

  }
  if (first_hit) *first_hit = res[0];
  if (n_hits) *n_hits = res[1];
  e.stats.hits += res[1];
  if (assign_out && res[0] != ~0ull) return read_assignment(e, *it->second, seed, res[0], assign_out);
  return MG_OK;
}

int mg_keccak256(const uint8_t* msgs, const uint32_t* lens, uint64_t n, uint8_t* out32) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  if (!e.init) return set_err(MG_E_NOTINIT, "mg_init not called");
  if (n == 0) return MG_OK;
  std::vector<uint64_t> offs(n);
  uint64_t tot = 0;
  for (uint64_t i = 0; i < n; i++) {
    offs[i] = tot;
    tot += lens[i];
  }
  uint8_t *d_msgs = nullptr, *d_out = nullptr;
  uint64_t* d_offs = nullptr;
  uint32_t* d_lens = nullptr;
  HIPCHK(hipMalloc((void**)&d_msgs, std::max<uint64_t>(tot, 1)));
  HIPCHK(hipMalloc((void**)&d_offs, n * 8));
  HIPCHK(hipMalloc((void**)&d_lens, n * 4));
  HIPCHK(hipMalloc((void**)&d_out, n * 32));
  if (tot) HIPCHK(hipMemcpy(d_msgs, msgs, tot, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_offs, offs.data(), n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_lens, lens, n * 4, hipMemcpyHostToDevice));
  const uint32_t block = 256;
  const uint32_t grid = (uint32_t)((n + block - 1) / block);
  HIPCHK(hipEventRecord(e.ev0, e.stream));
  hipLaunchKernelGGL(k_keccak, dim3(grid), dim3(block), 0, e.stream, d_msgs, d_offs, d_lens, n, d_out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e.ev1, e.stream));
  HIPCHK(hipEventSynchronize(e.ev1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e.ev0, e.ev1));
  e.stats.launches++;
  e.stats.last_kernel_ms = ms;
  e.stats.kernel_ms_total += ms;
  HIPCHK(hipMemcpy(out32, d_out, n * 32, hipMemcpyDeviceToHost));
  (void)hipFree(d_msgs);
  (void)hipFree(d_offs);
  (void)hipFree(d_lens);
  (void)hipFree(d_out);
  return MG_OK;
}

int mg_stats(mg_stats_t* out) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  *out = e.stats;
  out->jit_refused = jit_refused_total() - e.refused_base;
  return MG_OK;
}

int mg_stats_reset(void) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  mg_stats_t keep = e.stats;
  std::memset(&e.stats, 0, sizeof(e.stats));
  e.stats.device = keep.device;
  e.stats.cu_count = keep.cu_count;
  e.stats.clock_mhz = keep.clock_mhz;
  e.stats.n_devices = keep.n_devices;
  e.refused_base = jit_refused_total();
  return MG_OK;
}

int mg_dev_alloc(size_t bytes, void** dptr) {
  OnDevice od_(E());
  HIPCHK(hipMalloc(dptr, std::max<size_t>(bytes, 1)));
  return MG_OK;
}
int mg_dev_free(void* dptr) {
  HIPCHK(hipFree(dptr));
  return MG_OK;
}
int mg_dev_upload(void* dptr, const void* src, size_t bytes) {
  HIPCHK(hipMemcpy(dptr, src, bytes, hipMemcpyHostToDevice));
  return MG_OK;
}
int mg_dev_download(void* dst, const void* dptr, size_t bytes) {
  HIPCHK(hipMemcpy(dst, dptr, bytes, hipMemcpyDeviceToHost));
  return MG_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// JIT-specialised kernels
// ---------------------------------------------------------------------------
namespace mg {

// `nblk` is the kernel's grid-size argument (the JIT kernels read no dispatch packet)
static uint32_t jit_grid(const Engine& e, uint64_t count) {
  const uint64_t want = (count + 255) / 256;
  // MYTHGPU_JIT_BPC (default 64) 256-lane blocks per CU, i.e. 64 waves per SIMD over the
  // launch, whatever the occupancy (`nb`, unused here: the API answers 4 blocks/CU for a
  // 52-VGPR kernel the hardware runs 8 deep); the waves loop over aligned index groups.  Fewer
  // blocks leave a tail where the oldest waves of each SIMD have finished (16/CU: C4 -8 %, C5 -3 %,
  // C2 -2 %); more paid per-block start-up and the end-of-block publish, until the block's hits
  // went to a count stripe with no barrier (profiles/r03_ab_bpc_*.jsonl: 64 vs 32 per CU, kernel
  // time C2 -2.0 %, C4 -0.9 %, C1 -1.1 %, C3 -0.8 %; before the stripes C3 was 17 % slower at 64).
  // Launches past 2^29 candidates take 128 per CU (each wave still sweeps ~128 groups): the C2 step
  // of 2^30, 64 -> 128 per CU: +1.3 %, 32: -2.5 % (profiles/r03_ab_bpc_2p30.jsonl)
  static const int bpc_env = [] {
    const char* g = getenv("MYTHGPU_JIT_BPC");
    return g ? std::max(1, atoi(g)) : 0;
  }();
  // Small launches: every wave still sweeps at least MYTHGPU_JIT_MIN_GROUPS (default 16) groups of
  // 64 candidates, so its start-up (lane key, dictionary staging) and its end-of-wave publish are
  // amortised — at 64 blocks per CU a 2^24 launch gave each wave 4 groups (C2 60 G/s against 175
  // at 2^28, profiles/r03_config_sweeps.jsonl)
  static const uint64_t min_groups = [] {
    const char* g = getenv("MYTHGPU_JIT_MIN_GROUPS");
    return g ? (uint64_t)std::max(0, atoi(g)) : 16ull;
  }();
  uint64_t bpc = bpc_env ? (uint64_t)bpc_env : (count > (1ull << 29) ? 128u : 64u);
  if (!bpc_env && min_groups) {
    const uint64_t waves_cu = std::max<uint64_t>(1, ((count + 63) / 64) / (min_groups * (uint64_t)std::max(e.cu_count, 1)));
    bpc = std::max<uint64_t>(1, std::min(bpc, waves_cu / 4));
  }
  const uint64_t cap = (uint64_t)std::max(e.cu_count, 1) * bpc;
  return (uint32_t)std::max<uint64_t>(1, std::min(want, cap));
}

static int jit_launch_async(Engine& e, hipFunction_t f, int nb, uint64_t count, void** args, uint32_t& nblk) {
  (void)nb;
  const uint32_t grid = jit_grid(e, count);
  nblk = grid;
  HIPCHK(hipEventRecord(e.ev0, e.stream));
  HIPCHK(hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, e.stream, args, nullptr));
  HIPCHK(hipEventRecord(e.ev1, e.stream));
  return MG_OK;
}

static int jit_launch(Engine& e, hipFunction_t f, int nb, uint64_t count, void** args, uint32_t& nblk) {
  int rc = jit_launch_async(e, f, nb, count, args, nblk);
  if (rc) return rc;
  return launch_wait(e, e.stats, count);
}

// the JIT kernel `h` on device d: the primary's code object loaded there on first use
static int jit_on(Engine& d, const DevJit& pj, uint64_t h, DevJit** out) {
  auto it = d.jits.find(h);
  if (it != d.jits.end()) {
    *out = it->second.get();
    return MG_OK;
  }
  auto j = std::make_unique<DevJit>();
  HIPCHK(hipModuleLoadData(&j->mod, pj.code.data()));
  if (pj.fsearch) HIPCHK(hipModuleGetFunction(&j->fsearch, j->mod, "mgj_search"));
  j->nb_search = pj.nb_search;
  j->prog = pj.prog;
  j->gen = pj.gen;
  *out = j.get();
  d.jits[h] = std::move(j);
  return MG_OK;
}

}  // namespace mg

extern "C" {

int mg_program_jit_source(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words, int compile,
                          char* buf, size_t cap, size_t* out_len) {
  Lowered low;
  std::string err;
  int rc = lower_program(ssa, len, low, err);
  if (rc) return set_err(rc, err);
  std::vector<GenSpec> specs;
  std::vector<uint32_t> consts;
  if (gen_blob) {
    rc = parse_gen(low, gen_blob, gen_words, specs, consts, err);
    if (rc) return set_err(rc, err);
  }
  Lowered sp;
  // the same specialisation mg_gen_load / mg_jit_compile use (search: watch list dropped)
  rc = specialize_program(low, gen_blob ? &specs : nullptr, gen_blob ? &consts : nullptr, sp, err,
                          /*keep_watch=*/gen_blob == nullptr);
  if (rc) return set_err(rc, err);
  const std::string src = gen_blob ? jit_source(sp, &specs, &consts, JIT_SEARCH)
                                   : jit_source(sp, nullptr, nullptr, JIT_EVAL | ((compile & 2) ? JIT_EVAL_TILED : 0u));
  if (out_len) *out_len = src.size();
  if (buf && cap) {
    const size_t n = std::min(cap - 1, src.size());
    std::memcpy(buf, src.data(), n);
    buf[n] = 0;
  }
  if (compile & 1) {
    std::vector<char> code;
    std::string log;
    rc = jit_compile(src, code, log);
    if (rc) return set_err(rc, "JIT compile failed: " + log.substr(0, 4000));
  }
  return MG_OK;
}

int mg_program_jit_asm(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words, int compile,
                       char* buf, size_t cap, size_t* out_len) {
  Lowered low;
  std::string err;
  int rc = lower_program(ssa, len, low, err);
  if (rc) return set_err(rc, err);
  std::vector<GenSpec> specs;
  std::vector<uint32_t> consts;
  if (gen_blob) {
    rc = parse_gen(low, gen_blob, gen_words, specs, consts, err);
    if (rc) return set_err(rc, err);
  }
  Lowered sp;
  // with a generator: the search + gen kernels; without: the eval kernel (watch rows kept)
  rc = gen_blob ? specialize_program(low, &specs, &consts, sp, err, /*keep_watch=*/false)
                : specialize_program(low, nullptr, nullptr, sp, err);
  if (rc) return set_err(rc, err);
  std::string src;
  rc = jit_asm_source(sp, specs, consts, gen_blob ? (JIT_SEARCH | JIT_GEN) : (JIT_EVAL | ((compile & 2) ? JIT_EVAL_TILED : 0u)),
                      src, err);
  if (rc) return set_err(rc, "JIT assembly tier: " + err);
  if (out_len) *out_len = src.size();
  if (buf && cap) {
    const size_t n = std::min(cap - 1, src.size());
    std::memcpy(buf, src.data(), n);
    buf[n] = 0;
  }
  if (compile & 1) {
    std::vector<char> code;
    std::string log;
    rc = jit_compile(src, code, log);
    if (rc) return set_err(rc, "JIT assembly failed: " + log.substr(0, 4000));
  }
  return MG_OK;
}

int mg_collective_kind(void) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  if (!e.init) return set_err(MG_E_NOTINIT, "mg_init first");
  OnDevice od_(e);
  if (!collective_mode()) return 0;
  return rccl_ready() ? 1 : 0;
}

int mg_code_object_check(const void* code, size_t len, uint32_t* kernels, uint32_t* max_private_bytes,
                         uint32_t* max_group_bytes, uint32_t* dynamic_stack) {
  CodeObjectInfo ci;
  std::string err;
  if (int rc = code_object_info(code, len, ci, err)) return set_err(rc, err);
  if (kernels) *kernels = ci.kernels;
  if (max_private_bytes) *max_private_bytes = ci.max_private_bytes;
  if (max_group_bytes) *max_group_bytes = ci.max_group_bytes;
  if (dynamic_stack) *dynamic_stack = ci.dynamic_stack ? 1u : 0u;
  // the gate's verdict, not counted as a refusal of a JIT request
  std::string why;
  if (int rc = code_object_gate(ci, why)) return set_err(rc, why);
  return MG_OK;
}

int mg_jit_compile(uint64_t prog, uint64_t gen, uint64_t* jit_handle) { return mg_jit_compile_ex(prog, gen, 0, jit_handle); }

int mg_jit_helper_pid(void) { return jit_helper_pid(); }

int mg_cache_clear(void) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  e.lower_cache.clear();
  e.lower_order.clear();
  e.spec_cache.clear();
  e.spec_order.clear();
  std::lock_guard<std::mutex> jl(e.jit_mu);
  e.code_cache.lru.clear();
  e.code_cache.idx.clear();
  return MG_OK;
}

}  // extern "C"

namespace mg {

// load a code object as a DevJit (any thread: HIP module calls are thread-safe)
static int load_jit(const std::vector<char>& code, const JitTicket& t, double compile_ms, std::unique_ptr<DevJit>& out) {
  auto j = std::make_unique<DevJit>();
  j->code = code;
  HIPCHK(hipModuleLoadData(&j->mod, code.data()));
  int nb = 0;
  auto fn = [&](hipFunction_t* f, const char* name) -> int {
    if (hipModuleGetFunction(f, j->mod, name) != hipSuccess) {
      (void)hipModuleUnload(j->mod);
      return set_err(MG_E_HIP, std::string("JIT module has no ") + name);
    }
    return MG_OK;
  };
  if (t.has_gen) {
    if (int rc = fn(&j->fsearch, "mgj_search")) return rc;
    if (t.flags & MG_JIT_GEN_VERDICTS)
      if (int rc = fn(&j->fgen, "mgj_gen")) return rc;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, j->fsearch, 256, 0) == hipSuccess && nb > 0)
      j->nb_search = nb;
  } else {
    if (int rc = fn(&j->feval, "mgj_eval")) return rc;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, j->feval, 256, 0) == hipSuccess && nb > 0)
      j->nb_eval = nb;
  }
  j->prog = t.prog;
  j->gen = t.gen;
  j->compile_ms = compile_ms;
  j->asm_tier = (t.flags & MG_JIT_ASM) != 0;
  j->tiled = !t.has_gen && (t.flags & MG_JIT_SOA_TILED) != 0;
  out = std::move(j);
  return MG_OK;
}

// The tier of a verdict-only eval kernel (batched Model.eval) when the caller names none.  Both tiers
// are HBM-bound at different occupancies: on a small program LLVM's O3 kernel runs 8 waves per SIMD
// and beats the first tier's 4 (C2 token_transfer_underflow: O3 0.80 of HBM against 0.72), on a
// large one both run 2 waves and the first tier's row queue and instruction count win (C4
// walletlibrary_kill: first tier 0.71-0.73 against O3 0.49-0.52; BENCH_r05 roofline_eval,
// profiles/r06_eval_tiers.jsonl).  So the first tier's own register count decides: its kernel is
// kept when it runs at most 3 waves per SIMD (more than 128 VGPRs), else the O3 kernel is compiled.
// MYTHGPU_JIT_EVAL_TIER=o3|asm fixes the tier; MYTHGPU_JIT_EVAL_AUTO_VGPRS moves the threshold.
static int eval_tier_env() {
  static const int v = [] {
    const char* w = getenv("MYTHGPU_JIT_EVAL_TIER");
    if (!w) return 0;
    return std::string(w) == "o3" ? 1 : std::string(w) == "asm" ? 2 : 0;
  }();
  return v;
}

static bool eval_tier_pick_asm(const std::string& asm_src) {
  static const int thr = [] {
    const char* c = getenv("MYTHGPU_JIT_EVAL_AUTO_VGPRS");
    return c ? atoi(c) : 128;
  }();
  const size_t at = asm_src.find(".amdhsa_next_free_vgpr ");
  if (at == std::string::npos) return true;
  return atoi(asm_src.c_str() + at + 23) > thr;
}

static void jit_worker_main(Engine* ep, int device, int lane) {
  Engine& e = *ep;
  (void)hipSetDevice(device);
  std::unique_lock<std::mutex> lk(e.jit_mu);
  auto& queue = e.jit_queue[lane ? 1 : 0];
  for (;;) {
    e.jit_cv.wait(lk, [&] { return e.jit_stop || !queue.empty(); });
    if (e.jit_stop) {
      e.jit_workers--;
      e.jit_done_cv.notify_all();
      return;
    }
    std::shared_ptr<JitTicket> t = queue.front();
    queue.pop_front();
    if (t->cancelled) continue;
    lk.unlock();
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t kernels = t->has_gen ? (JIT_SEARCH | ((t->flags & MG_JIT_GEN_VERDICTS) ? JIT_GEN : 0u))
                                        : (JIT_EVAL | ((t->flags & MG_JIT_SOA_TILED) ? JIT_EVAL_TILED : 0u));
    std::string src, asm_err;
    int asm_rc = MG_OK;
    if (t->flags & MG_JIT_ASM) {
      // the first tier: assembly straight from the specialised program (jit_asm.cpp)
      asm_rc = jit_asm_source(t->low, t->specs, t->consts, kernels, src, asm_err);
      if (asm_rc == MG_OK && t->auto_eval && !eval_tier_pick_asm(src)) {
        t->flags &= ~MG_JIT_ASM;
        src = jit_source(t->low, nullptr, nullptr, kernels);
      }
      if (asm_rc != MG_OK && t->asm_fallback) {  // chosen by default: the O3 kernel instead
        // (not at -O0: LLVM's -O0 kernel for a VMTests read-back kept 52 KB of stack per lane in a
        // dynamic stack and faulted on the GPU; -O1 compiled no faster than -O3)
        t->flags &= ~MG_JIT_ASM;
        asm_rc = MG_OK;
        src = jit_source(t->low, nullptr, nullptr, kernels);
      }
    } else {
      src = t->has_gen ? jit_source(t->low, &t->specs, &t->consts, kernels) : jit_source(t->low, nullptr, nullptr, kernels);
    }
    const auto t_src = std::chrono::steady_clock::now();
    if (asm_rc != MG_OK) {
      lk.lock();
      t->rc = asm_rc;
      t->err = "JIT assembly tier: " + asm_err;
      t->state = JitTicket::FAILED;
      e.jit_done_cv.notify_all();
      continue;
    }
    std::unique_ptr<DevJit> j;
    std::vector<char> code;
    lk.lock();
    // the same source compiling on the other lane: wait for it, then take it from the cache
    e.jit_done_cv.wait(lk, [&] { return e.jit_stop || !e.jit_inflight.count(src); });
    if (CodeCache::Entry* en = e.code_cache.find_entry(src)) {
      code = en->code;
      if (en->hold) {  // resident module: no load
        j = std::make_unique<DevJit>();
        j->code = en->code;
        j->hold = en->hold;
        j->mod = en->hold->mod;
        j->fsearch = en->fsearch;
        j->feval = en->feval;
        j->fgen = en->fgen;
        j->nb_search = en->nb_search;
        j->nb_eval = en->nb_eval;
        j->prog = t->prog;
        j->gen = t->gen;
        j->asm_tier = (t->flags & MG_JIT_ASM) != 0;
        j->tiled = !t->has_gen && (t->flags & MG_JIT_SOA_TILED) != 0;
        j->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      }
    }
    // a search that ended while this request waited: nothing to compile for it
    const bool skip = !j && code.empty() && t->cancelled;
    const bool owner = !j && code.empty() && !skip;
    if (owner) e.jit_inflight.insert(src);
    lk.unlock();
    int rc = MG_OK;
    std::string log;
    bool compiled = false, from_disk = false;
    if (owner) {
      rc = jit_compile(src, code, log, &from_disk);
      compiled = rc == MG_OK;
    }
    if (skip) {
      lk.lock();
      t->state = JitTicket::FAILED;
      t->rc = MG_E_INVALID;
      t->err = "cancelled";
      e.jit_done_cv.notify_all();
      continue;
    }
    std::string err;
    const auto t_comp = std::chrono::steady_clock::now();
    if (rc != MG_OK) {
      err = "JIT compile failed: " + log.substr(0, 4000);
    } else if (!j) {
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      rc = load_jit(code, *t, ms, j);
      if (getenv("MYTHGPU_JIT_TIMING")) {
        auto d = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "mythgpu jit worker (%s): queued %.2f ms, source %.2f ms, compile %.2f ms, module load %.2f ms\n",
                (t->flags & MG_JIT_ASM) ? "asm" : "o3", d(t->submitted, t0), d(t0, t_src), d(t_src, t_comp),
                d(t_comp, std::chrono::steady_clock::now()));
      }
      if (rc != MG_OK && from_disk) {
        // a disk-cache entry that passes the header checks but does not load (a truncated write
        // renamed on a full disk, a runtime upgrade without a rebuild): drop it and compile once
        jit_disk_evict(src);
        code.clear();
        rc = jit_compile(src, code, log, &from_disk);
        ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (rc == MG_OK) rc = load_jit(code, *t, ms, j);
        else g_err = "JIT compile failed: " + log.substr(0, 4000);
      }
      if (rc != MG_OK) {
        err = g_err;
      } else {
        // the cache keeps the module loaded for the next request of the same source
        j->hold = std::make_shared<ModHold>(j->mod);
        lk.lock();
        if (compiled) e.code_cache.insert(src, std::vector<char>(code));
        if (CodeCache::Entry* en = e.code_cache.find_entry(src)) {
          if (!en->hold) {
            en->hold = j->hold;
            en->fsearch = j->fsearch;
            en->feval = j->feval;
            en->fgen = j->fgen;
            en->nb_search = j->nb_search;
            en->nb_eval = j->nb_eval;
          }
        }
        lk.unlock();
      }
    }
    lk.lock();
    if (owner) e.jit_inflight.erase(src);  // (waiters wake on the notify below)
    if (rc != MG_OK) {
      t->rc = rc;
      t->err = err;
      t->state = JitTicket::FAILED;
    } else if (t->cancelled) {
      release_jit(*j);
      t->state = JitTicket::FAILED;
      t->rc = MG_E_INVALID;
      t->err = "cancelled";
    } else {
      t->ready = std::move(j);
      t->state = JitTicket::DONE;
    }
    e.jit_done_cv.notify_all();
  }
}

// process exit with a compile in flight: stop the compile thread before the compiler
// library's static destructors run (registered after them, so it runs first)
static void jit_atexit() {
  wait_warm();
  Engine& e = E();
  std::unique_lock<std::mutex> jl(e.jit_mu);
  e.jit_stop = true;
  for (auto& q : e.jit_queue)
    for (auto& t : q) t->cancelled = true;
  for (auto& kv : e.tickets) kv.second->cancelled = true;
  e.jit_cv.notify_all();
  e.jit_done_cv.wait_for(jl, std::chrono::seconds(10), [&] { return e.jit_workers == 0; });
}

// caller holds e.mu
static int submit_jit(Engine& e, uint64_t prog, uint64_t gen, uint32_t flags, uint64_t* ticket) {
  DevProgram* p = find_prog(e, prog);
  if (!p) return set_err(MG_E_INVALID, "bad program handle");
  auto t = std::make_shared<JitTicket>();
  t->prog = prog;
  t->gen = gen;
  t->flags = flags;
  if (gen) {
    auto it = e.gens.find(gen);
    if (it == e.gens.end() || it->second->prog != prog) return set_err(MG_E_INVALID, "bad generator handle");
    // with a generator: the search kernel on its specialised program
    t->low = it->second->spec.low;
    t->specs = it->second->specs;
    t->consts = it->second->consts;
    t->has_gen = true;
  } else {
    // without: the eval kernel
    std::string err;
    int rc = specialize_program(p->low, nullptr, nullptr, t->low, err);
    if (rc) return set_err(rc, err);
    // watch rows (model read-back, batched term evaluation): the first tier's eval kernel stores them
    // from the values' registers (no SGPR spills; the O3 kernel's indexed row stores spill hundreds of
    // v_readlane / v_writelane on C4), and compiles in a few ms; O3 if the first tier refuses
    static const bool o3_env = [] {
      const char* w = getenv("MYTHGPU_JIT_WATCH_TIER");
      return w && std::string(w) == "o3";
    }();
    if (t->low.watch_words && !(flags & (MG_JIT_ASM | MG_JIT_O3)) && !o3_env) {
      t->flags |= MG_JIT_ASM;
      t->asm_fallback = true;
    }
    // verdicts only (batched Model.eval): the worker emits the first tier and keeps it for a program
    // whose kernel runs at <= 3 waves per SIMD, else compiles the O3 kernel (eval_tier_pick)
    if (!t->low.watch_words && !(flags & (MG_JIT_ASM | MG_JIT_O3)) && eval_tier_env() != 1) {
      t->flags |= MG_JIT_ASM;
      t->asm_fallback = true;
      t->auto_eval = eval_tier_env() == 0;
    }
  }
  const uint64_t h = e.next_handle++;
  std::lock_guard<std::mutex> jl(e.jit_mu);
  if (e.jit_workers == 0) {
    static std::once_flag once;
    std::call_once(once, [] {
      jit_compiler_preload();
      std::atexit(jit_atexit);
    });
    if (const char* c = getenv("MYTHGPU_JIT_CACHE")) e.code_cache.cap = std::max(1, atoi(c));
    // lane 0: O3 compiles; lanes 1 and 2 share the first tier's queue (and its two assembly helpers), so
    // a new search's assembly does not wait for one a finished search left in flight
    for (int lane = 0; lane < 3; lane++) std::thread(jit_worker_main, &e, e.device, lane).detach();
    e.jit_workers = 3;
  }
  e.tickets[h] = t;
  e.jit_queue[(t->flags & MG_JIT_ASM) ? 1 : 0].push_back(t);
  e.jit_cv.notify_all();
  *ticket = h;
  return MG_OK;
}

// caller holds e.mu; wait_ms < 0: until done.  A finished kernel moves into e.jits here.
static int poll_jit(Engine& e, uint64_t ticket, int64_t wait_ms, uint64_t* jit) {
  *jit = 0;
  std::shared_ptr<JitTicket> t;
  {
    std::unique_lock<std::mutex> jl(e.jit_mu);
    auto it = e.tickets.find(ticket);
    if (it == e.tickets.end()) return set_err(MG_E_INVALID, "bad JIT ticket");
    t = it->second;
    auto ready = [&] { return t->state != JitTicket::PENDING; };
    if (wait_ms < 0) e.jit_done_cv.wait(jl, ready);
    else if (wait_ms > 0) e.jit_done_cv.wait_for(jl, std::chrono::milliseconds(wait_ms), ready);
    if (t->state == JitTicket::PENDING) return MG_OK;
    e.tickets.erase(ticket);
  }
  if (t->state == JitTicket::FAILED) return set_err(t->rc ? t->rc : MG_E_HIP, t->err);
  if (!e.progs.count(t->prog) || (t->has_gen && !e.gens.count(t->gen))) {
    release_jit(*t->ready);
    return set_err(MG_E_INVALID, "program or generator freed before its JIT kernel was ready");
  }
  const uint64_t h = e.next_handle++;
  e.jits[h] = std::move(t->ready);
  *jit = h;
  return MG_OK;
}

}  // namespace mg

extern "C" {

int mg_jit_compile_ex(uint64_t prog, uint64_t gen, uint32_t flags, uint64_t* jit_handle) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  uint64_t ticket = 0;
  int rc = submit_jit(e, prog, gen, flags, &ticket);
  if (rc) return rc;
  return poll_jit(e, ticket, -1, jit_handle);
}

int mg_jit_compile_async(uint64_t prog, uint64_t gen, uint32_t flags, uint64_t* ticket) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  return submit_jit(e, prog, gen, flags, ticket);
}

int mg_jit_poll(uint64_t ticket, int32_t wait_ms, uint64_t* jit_handle) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  return poll_jit(e, ticket, wait_ms, jit_handle);
}

int mg_jit_cancel(uint64_t ticket) {
  Engine& e = E();
  std::lock_guard<std::mutex> jl(e.jit_mu);
  auto it = e.tickets.find(ticket);
  if (it == e.tickets.end()) return set_err(MG_E_INVALID, "bad JIT ticket");
  std::shared_ptr<JitTicket> t = it->second;
  e.tickets.erase(it);
  if (t->state == JitTicket::PENDING) {
    t->cancelled = true;  // the worker drops it (before compiling if still queued)
  } else if (t->state == JitTicket::DONE && t->ready) {
    release_jit(*t->ready);
    t->ready.reset();
  }
  return MG_OK;
}

int mg_jit_info(uint64_t jit, double* compile_ms, int* blocks_per_cu) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.jits.find(jit);
  if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
  if (compile_ms) *compile_ms = it->second->compile_ms;
  if (blocks_per_cu) *blocks_per_cu = it->second->nb_search;
  return MG_OK;
}

int mg_jit_layout(uint64_t jit, uint32_t* flags, uint32_t* coord_words, uint32_t* watch_words) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.jits.find(jit);
  if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
  const DevJit& j = *it->second;
  DevProgram* p = find_prog(e, j.prog);
  if (!p) return set_err(MG_E_INVALID, "jit program was freed");
  if (flags) *flags = (j.asm_tier ? MG_JIT_ASM : 0u) | (j.tiled ? MG_JIT_SOA_TILED : 0u) | (j.fgen ? MG_JIT_GEN_VERDICTS : 0u);
  if (coord_words) *coord_words = p->low.coord_words;
  if (watch_words) *watch_words = p->low.watch_words;
  return MG_OK;
}

int mg_jit_free(uint64_t jit) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.jits.find(jit);
  if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
  release_jit(*it->second);
  e.jits.erase(it);
  for (size_t i = 1; i < g_devs.size(); i++) {
    auto q = g_devs[i]->jits.find(jit);
    if (q == g_devs[i]->jits.end()) continue;
    (void)hipSetDevice(g_devs[i]->device);
    release_jit(*q->second);
    g_devs[i]->jits.erase(q);
  }
  if (g_devs.size() > 1) (void)hipSetDevice(e.device);
  return MG_OK;
}

int mg_jit_search(uint64_t jit, uint64_t seed, uint64_t start, uint64_t count, uint32_t flags, uint64_t* first_hit,
                  uint64_t* n_hits, uint32_t* assign_out) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.jits.find(jit);
  if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
  DevJit& j = *it->second;
  DevProgram* p = find_prog(e, j.prog);
  auto git = e.gens.find(j.gen);
  if (!p || git == e.gens.end() || !j.fsearch) return set_err(MG_E_INVALID, "jit was not compiled for search");
  // the search kernel counts each wave's groups in 32 bits (jit.cpp): at most 2^52 candidates per call
  if (count > (1ull << 52)) return set_err(MG_E_INVALID, "mg_jit_search: more than 2^52 candidates in one call");
  uint64_t sk = seed_lane_key(seed), sg = seed_group_key(seed);
  unsigned long long res[2] = {~0ull, 0ull};
  if (split_over_devices(count)) {  // as mg_search: one group-aligned slice per device, host min/sum
    const uint32_t nd = (uint32_t)g_devs.size();
    std::vector<uint64_t> st(nd), ct(nd);
    mg_split_range(start, count, nd, st.data(), ct.data());
    // kernel arguments must outlive the asynchronous launches
    struct A {
      const uint32_t* gconsts;
      uint64_t start, count, sk, sg;
      unsigned long long* hit;
      uint32_t flags, nblk;
    };
    std::vector<A> a(nd);
    int rc = MG_OK;
    const bool coll = rccl_ready();  // the exchange as one RCCL all-reduce(min) (MYTHGPU_COLLECTIVE)
    for (uint32_t d = 0; d < nd && rc == MG_OK; d++) {
      if (!ct[d]) continue;
      Engine& de = *g_devs[d];
      HIPCHK(hipSetDevice(de.device));
      DevGen& dg = *de.gens.at(j.gen);
      if ((rc = ensure_gen_on(de, dg))) break;
      DevJit* dj = &j;
      if (d > 0 && (rc = jit_on(de, j, jit, &dj))) break;
      if ((rc = arm_hits(de))) break;
      a[d] = A{dg.d_consts, st[d], ct[d], sk, sg, de.d_hit, flags | (de.sys_scope ? MG_SEARCH_SYSTEM_SCOPE : 0u), 0};
      void* args[] = {&a[d].gconsts, &a[d].start, &a[d].count, &a[d].sk, &a[d].sg, &a[d].hit, &a[d].flags, &a[d].nblk};
      const uint64_t lanes = (st[d] + ct[d]) - (st[d] & ~63ull);
      // hipModuleLaunchKernel copies the argument values at the call (nblk is set before it)
      rc = jit_launch_async(de, dj->fsearch, dj->nb_search, lanes, args, a[d].nblk);
      if (rc == MG_OK && !coll) rc = fetch_hits(de);
    }
    if (rc == MG_OK && coll) rc = rccl_fetch(ct);
    for (uint32_t d = 0; d < nd; d++) {
      if (!ct[d]) continue;
      Engine& de = *g_devs[d];
      (void)hipSetDevice(de.device);
      unsigned long long r[2];
      if (rc == MG_OK) rc = collect_hits(de, e.stats, ct[d], r);
      if (rc == MG_OK) {
        res[0] = std::min(res[0], r[0]);
        res[1] += r[1];
      }
    }
    HIPCHK(hipSetDevice(e.device));
    if (rc) return rc;
  } else {
    const uint32_t* gconsts = git->second->d_consts;
    unsigned long long* hitp = e.d_hit;
    uint32_t nblk = 0;
    void* args[] = {&gconsts, &start, &count, &sk, &sg, &hitp, &flags, &nblk};
    // one wave per aligned 64-index group
    const uint64_t lanes = (start + count) - (start & ~63ull);
    int rc = arm_hits(e);
    if (!rc) rc = jit_launch_async(e, j.fsearch, j.nb_search, lanes, args, nblk);
    // MYTHGPU_COLLECTIVE=rccl-force on one device: the same all-reduce over a one-rank communicator
    if (!rc && collective_mode() == 2 && g_devs.size() == 1 && rccl_ready()) rc = rccl_first_hit_min();
    if (!rc) rc = fetch_hits(e);
    if (!rc) rc = collect_hits(e, e.stats, count, res);
    if (rc) return rc;
  }
  if (first_hit) *first_hit = res[0];
  if (n_hits) *n_hits = res[1];
  e.stats.hits += res[1];
  if (assign_out && res[0] != ~0ull) return read_assignment(e, *git->second, seed, res[0], assign_out);
  return MG_OK;
}

int mg_jit_search_many(uint64_t jit, uint32_t n, const uint64_t* seeds, const uint64_t* starts, const uint64_t* counts,
                       uint32_t flags, uint64_t* first_hits, uint64_t* n_hits) {
  if (n == 0) return MG_OK;
  if (!seeds || !starts || !counts || !first_hits || !n_hits) return set_err(MG_E_INVALID, "mg_jit_search_many: null array");
  Engine& e = E();
  bool split = false;
  for (uint32_t q = 0; q < n; q++) split = split || split_over_devices(counts[q]);
  if (split) {  // several devices per launch: one mg_jit_search after the other
    for (uint32_t q = 0; q < n; q++) {
      const int rc = mg_jit_search(jit, seeds[q], starts[q], counts[q], flags, first_hits + q, n_hits + q, nullptr);
      if (rc) return rc;
    }
    return MG_OK;
  }
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.jits.find(jit);
  if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
  DevJit& j = *it->second;
  auto git = e.gens.find(j.gen);
  if (!find_prog(e, j.prog) || git == e.gens.end() || !j.fsearch) return set_err(MG_E_INVALID, "jit was not compiled for search");
  for (uint32_t q = 0; q < n; q++)
    if (counts[q] > (1ull << 52)) return set_err(MG_E_INVALID, "mg_jit_search_many: more than 2^52 candidates in one launch");
  if (!e.d_hitmany) {
    HIPCHK(hipMalloc((void**)&e.d_hitmany, (size_t)kManySlots * kHitAlloc * sizeof(unsigned long long)));
    HIPCHK(hipHostMalloc((void**)&e.h_hitmany, 2 * (size_t)kManySlots * kHitAlloc * sizeof(unsigned long long),
                         hipHostMallocDefault));
    std::memset(e.h_hitmany, 0, 2 * (size_t)kManySlots * kHitAlloc * sizeof(unsigned long long));
    for (uint32_t q = 0; q < kManySlots; q++) e.h_hitmany[(size_t)q * kHitAlloc] = ~0ull;  // armed; peer count 0
    for (int q = 0; q < kManyStreams; q++) {
      HIPCHK(hipStreamCreateWithFlags(&e.xs[q], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&e.xev[q], hipEventDisableTiming));
    }
  }
  const uint32_t* gconsts = git->second->d_consts;
  for (uint32_t b0 = 0; b0 < n; b0 += kManySlots) {
    const uint32_t m = std::min<uint32_t>(kManySlots, n - b0);
    const size_t bytes = (size_t)m * kHitAlloc * sizeof(unsigned long long);
    unsigned long long* back = e.h_hitmany + (size_t)kManySlots * kHitAlloc;
    // arm m slots with one copy on the engine stream; the launch streams wait for it
    HIPCHK(hipEventRecord(e.ev0, e.stream));
    HIPCHK(hipMemcpyAsync(e.d_hitmany, e.h_hitmany, bytes, hipMemcpyHostToDevice, e.stream));
    HIPCHK(hipEventRecord(e.ev2, e.stream));
    for (int q = 0; q < kManyStreams; q++) HIPCHK(hipStreamWaitEvent(e.xs[q], e.ev2, 0));
    uint64_t total = 0;
    for (uint32_t q = 0; q < m; q++) {
      uint64_t start = starts[b0 + q], count = counts[b0 + q];
      uint64_t sk = seed_lane_key(seeds[b0 + q]), sg = seed_group_key(seeds[b0 + q]);
      unsigned long long* hitp = e.d_hitmany + (size_t)q * kHitAlloc;
      uint32_t f = flags;
      const uint64_t lanes = (start + count) - (start & ~63ull);
      uint32_t nblk = jit_grid(e, lanes);
      void* args[] = {&gconsts, &start, &count, &sk, &sg, &hitp, &f, &nblk};
      total += count;
      if (count == 0) continue;
      // hipModuleLaunchKernel copies the argument values at the call
      const hipError_t le = hipModuleLaunchKernel(j.fsearch, nblk, 1, 1, 256, 1, 1, 0, e.xs[q % kManyStreams], args, nullptr);
      if (le != hipSuccess) {  // the launches already queued finish before the slots are reused
        for (int s2 = 0; s2 < kManyStreams; s2++) (void)hipStreamSynchronize(e.xs[s2]);
        return set_err(MG_E_HIP, std::string("mg_jit_search_many: ") + hipGetErrorString(le));
      }
    }
    for (int q = 0; q < kManyStreams; q++) {
      HIPCHK(hipEventRecord(e.xev[q], e.xs[q]));
      HIPCHK(hipStreamWaitEvent(e.stream, e.xev[q], 0));
    }
    HIPCHK(hipEventRecord(e.ev1, e.stream));
    HIPCHK(hipMemcpyAsync(back, e.d_hitmany, bytes, hipMemcpyDeviceToHost, e.stream));
    HIPCHK(hipEventRecord(e.ev2, e.stream));
    HIPCHK(hipEventSynchronize(e.ev2));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e.ev0, e.ev1));
    e.stats.launches += m;
    e.stats.last_kernel_ms = ms;  // the batch's arm .. last kernel
    e.stats.kernel_ms_total += ms;
    e.stats.candidates += total;
    e.stats.last_candidates = total;
    for (uint32_t q = 0; q < m; q++) {
      const unsigned long long* r = back + (size_t)q * kHitAlloc;
      uint64_t h = r[1];
      for (uint32_t t = 1; t <= kHitStripes; t++) h += r[kHitStride * t];
      first_hits[b0 + q] = counts[b0 + q] ? r[0] : ~0ull;
      n_hits[b0 + q] = counts[b0 + q] ? h : 0;
      e.stats.hits += n_hits[b0 + q];
    }
  }
  return MG_OK;
}

int mg_jit_verdicts(uint64_t jit, uint64_t seed, uint64_t start, uint64_t n, uint8_t* verdict_out) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.jits.find(jit);
  if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
  DevJit& j = *it->second;
  auto git = e.gens.find(j.gen);
  if (git == e.gens.end() || !j.fgen) return set_err(MG_E_INVALID, "jit was not compiled with MG_JIT_GEN_VERDICTS");
  if (n == 0) return MG_OK;
  uint8_t* d_ver = nullptr;
  HIPCHK(hipMalloc((void**)&d_ver, n));
  const uint32_t* gconsts = git->second->d_consts;
  uint64_t sk = seed_lane_key(seed), sg = seed_group_key(seed);
  uint32_t nblk = 0;
  void* args[] = {&gconsts, &start, &n, &sk, &sg, &d_ver, &nblk};
  const uint64_t lanes = (start + n) - (start & ~63ull);
  int rc = jit_launch(e, j.fgen, j.nb_search, lanes, args, nblk);
  if (rc == MG_OK) {
    hipError_t he = hipMemcpy(verdict_out, d_ver, n, hipMemcpyDeviceToHost);
    if (he != hipSuccess) rc = set_err(MG_E_HIP, hipGetErrorString(he));
  }
  (void)hipFree(d_ver);
  return rc;
}

int mg_jit_eval_dev(uint64_t jit, const uint32_t* d_soa, uint64_t n, uint8_t* d_verdict, uint32_t* d_watch) {
  Engine& e = E();
  std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
  auto it = e.jits.find(jit);
  if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
  DevJit& j = *it->second;
  if (!j.feval) return set_err(MG_E_INVALID, "jit was not compiled for eval (compile with gen = 0)");
  if (j.asm_tier && n >= (1ull << 30))
    return set_err(MG_E_UNSUPPORTED, "the first tier's eval kernel takes fewer than 2^30 candidates per call");
  uint32_t nblk = 0;
  void* args[] = {&d_soa, &n, &d_verdict, &d_watch, &nblk};
  if (j.eval_cpb < 0) {
    CodeObjectInfo ci;
    std::string err;
    j.eval_cpb = (!j.code.empty() && code_object_info(j.code.data(), j.code.size(), ci, err) == MG_OK) ? (int)ci.eval_cpb : 0;
  }
  if (j.eval_cpb > 0) {  // one group per workgroup, no loop: the grid covers every candidate
    const uint64_t blocks = (n + (uint64_t)j.eval_cpb - 1) / (uint64_t)j.eval_cpb;
    if (blocks > 0xFFFFFFFFull) return set_err(MG_E_UNSUPPORTED, "eval launch too wide for a loop-free kernel");
    nblk = (uint32_t)blocks;
    HIPCHK(hipEventRecord(e.ev0, e.stream));
    HIPCHK(hipModuleLaunchKernel(j.feval, nblk, 1, 1, 256, 1, 1, 0, e.stream, args, nullptr));
    HIPCHK(hipEventRecord(e.ev1, e.stream));
    return launch_wait(e, e.stats, n);
  }
  return jit_launch(e, j.feval, j.nb_eval, n, args, nblk);
}

int mg_jit_eval(uint64_t jit, const uint32_t* soa, uint64_t n, uint8_t* verdict_out, uint32_t* watch_out) {
  Engine& e = E();
  DevProgram* p;
  bool tiled = false;
  {
    std::lock_guard<std::mutex> g(e.mu);
  OnDevice od_(e);
    auto it = e.jits.find(jit);
    if (it == e.jits.end()) return set_err(MG_E_INVALID, "bad jit handle");
    p = find_prog(e, it->second->prog);
    if (!p) return set_err(MG_E_INVALID, "jit program was freed");
    tiled = it->second->tiled;
  }
  if (n == 0) return MG_OK;
  // a tiled SoA (MG_JIT_SOA_TILED) holds ceil(n / 64) whole 64-candidate blocks
  const uint64_t soa_cols = tiled ? (n + 63) / 64 * 64 : n;
  const size_t soa_bytes = (size_t)std::max<uint32_t>(p->low.coord_words, 1) * soa_cols * 4;
  const size_t watch_bytes = (size_t)p->low.watch_words * n * 4;
  uint32_t *d_soa = nullptr, *d_watch = nullptr;
  uint8_t* d_ver = nullptr;
  // freed on every return, the early error returns of HIPCHK included
  struct Frees {
    void** p[3];
    ~Frees() {
      for (void** q : p)
        if (*q) (void)hipFree(*q);
    }
  } frees_{{(void**)&d_soa, (void**)&d_ver, (void**)&d_watch}};
  HIPCHK(hipMalloc((void**)&d_soa, soa_bytes));
  HIPCHK(hipMalloc((void**)&d_ver, n));
  if (watch_out && watch_bytes) HIPCHK(hipMalloc((void**)&d_watch, watch_bytes));
  if (p->low.coord_words) HIPCHK(hipMemcpy(d_soa, soa, (size_t)p->low.coord_words * soa_cols * 4, hipMemcpyHostToDevice));
  int rc = mg_jit_eval_dev(jit, d_soa, n, d_ver, d_watch);
  if (rc == MG_OK) {
    HIPCHK(hipMemcpy(verdict_out, d_ver, n, hipMemcpyDeviceToHost));
    if (d_watch) HIPCHK(hipMemcpy(watch_out, d_watch, watch_bytes, hipMemcpyDeviceToHost));
  }
  return rc;
}

}  // extern "C"
