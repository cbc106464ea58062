// INT32 VALU issue-rate microbenchmark for gfx950 (MI355X).
//
// Measures the wave64 issue cost of the integer VALU instructions the search
// kernel is made of, each as NCHAIN independent dependency chains per lane, at
// 1/2/4/8 waves per SIMD.  Cycles come from s_memtime inside the kernel (one
// tick = one shader cycle, MI355X_MICROARCH.md constants table), so the result
// does not depend on the clock the chip runs at; lane-ops/s use the event time.
// v_fma_f32 is included to calibrate against the guide's measured 2 cycles.
//
// Output: one JSON line per (op, waves/SIMD).  Pins the "peak" for roofline.frac.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_peak tools/valu_peak.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int ITERS = 1024;
constexpr int NCHAIN = 8;

enum Op {
  FMA_F32 = 0, ADD, XOR, LSHR, ADD_LIT, ADDC, SUBB, CND_VCC, CND_SGPR, CMP, MULLO, MULHI, MAD64, LSHLOR, ADD3,
  OR3, ALIGNBIT, BFE, PERM, NOPS
};
static const char* kNames[NOPS] = {
    "v_fma_f32", "v_add_u32", "v_xor_b32", "v_lshrrev_b32", "v_add_u32 (literal)", "v_add_co_u32+v_addc_co_u32",
    "v_sub_co_u32+v_subb_co_u32", "v_cndmask_b32 (vcc)", "v_cndmask_b32_e64 (sgpr mask)", "v_cmp_lt_u32_e64",
    "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_lshl_or_b32", "v_add3_u32", "v_or3_b32",
    "v_alignbit_b32", "v_bfe_u32", "v_perm_b32"};
static const int kInstr[NOPS] = {1, 1, 1, 1, 1, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};

template <int OP>
__global__ void __launch_bounds__(64) k_valu(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  uint32_t a[NCHAIN], b[NCHAIN];
  float f[NCHAIN];
#pragma unroll
  for (int c = 0; c < NCHAIN; c++) {
    a[c] = seed * (threadIdx.x + 1) + c;
    b[c] = seed ^ (c * 0x9E3779B9u + threadIdx.x);
    f[c] = (float)a[c];
  }
  const uint32_t k = seed | 1u;
  const float fk = 1.0001f;
  uint64_t m;  // lane mask in an SGPR pair
  asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(a[0]), "v"(b[0]));
  asm volatile("s_mov_b64 vcc, %0" ::"s"(m) : "vcc");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < NCHAIN; c++) {
      if constexpr (OP == FMA_F32) {
        asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(fk));
      } else if constexpr (OP == ADD) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == XOR) {
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == LSHR) {
        asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == ADD_LIT) {
        asm volatile("v_add_u32 %0, 0x9e3779b9, %0" : "+v"(a[c]));
      } else if constexpr (OP == ADDC) {
        uint64_t cy;
        asm volatile(
            "v_add_co_u32 %0, %2, %0, %3\n\t"
            "v_addc_co_u32 %1, %2, %1, %3, %2"
            : "+v"(a[c]), "+v"(b[c]), "=&s"(cy)
            : "v"(k));
      } else if constexpr (OP == SUBB) {
        uint64_t cy;
        asm volatile(
            "v_sub_co_u32 %0, %2, %0, %3\n\t"
            "v_subb_co_u32 %1, %2, %1, %3, %2"
            : "+v"(a[c]), "+v"(b[c]), "=&s"(cy)
            : "v"(k));
      } else if constexpr (OP == CND_VCC) {
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(b[c]) : "vcc");
      } else if constexpr (OP == CND_SGPR) {
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b[c]), "s"(m));
      } else if constexpr (OP == CMP) {
        uint64_t r;
        asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(r) : "v"(a[c]), "v"(b[c]));
        asm volatile("" ::"s"(r));
      } else if constexpr (OP == MULLO) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == MULHI) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == MAD64) {
        uint64_t acc = ((uint64_t)b[c] << 32) | a[c];
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=&s"(cy) : "v"(k), "v"(k));
        a[c] = (uint32_t)acc;
        b[c] = (uint32_t)(acc >> 32);
      } else if constexpr (OP == LSHLOR) {
        asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == ADD3) {
        asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == OR3) {
        asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == ALIGNBIT) {
        asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[c]) : "v"(b[c]));
      } else if constexpr (OP == BFE) {
        asm volatile("v_bfe_u32 %0, %0, 3, 17" : "+v"(a[c]));
      } else {
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b[c]), "v"(k));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < NCHAIN; c++) s ^= a[c] ^ b[c] ^ __float_as_uint(f[c]);
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(int cus, uint32_t* d, unsigned long long* dc, hipEvent_t e0, hipEvent_t e1, double ghz) {
  for (int wps : {1, 2, 4, 8}) {
    // one 64-thread block = one wave; cus*4*wps blocks put wps waves on every SIMD
    const int blocks = cus * 4 * wps;
    hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(64), 0, 0, d, dc, 7u);  // warm-up
    CHK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(64), 0, 0, d, dc, 7u + r);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> c(blocks);
    CHK(hipMemcpy(c.data(), dc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double mean = 0;
    for (auto x : c) mean += (double)x;
    mean /= blocks;
    const double s = ms * 1e-3 / reps;
    const double per_wave = (double)ITERS * NCHAIN * kInstr[OP];
    const double winstr = blocks * per_wave;
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_instr_per_simd\": %.3f, "
           "\"lane_ops_T_per_s\": %.3f, \"lane_ops_T_per_s_at_2p4GHz\": %.3f, \"us\": %.1f}\n",
           kNames[OP], wps, mean / (wps * per_wave), winstr * 64 / s / 1e12,
           cus * 4 * 64 * ghz * 1e9 / (mean / (wps * per_wave)) / 1e12, s * 1e6);
    fflush(stdout);
  }
}

template <int OP>
static void run_all(int cus, uint32_t* d, unsigned long long* dc, hipEvent_t e0, hipEvent_t e1, double ghz) {
  if constexpr (OP < NOPS) {
    run<OP>(cus, d, dc, e0, e1, ghz);
    run_all<OP + 1>(cus, d, dc, e0, e1, ghz);
  }
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double ghz = p.clockRate / 1e6;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_ghz_nominal\": %.3f}\n", p.gcnArchName, cus, ghz);
  uint32_t* d;
  unsigned long long* dc;
  CHK(hipMalloc(&d, (size_t)cus * 4 * 8 * 64 * 4));
  CHK(hipMalloc(&dc, (size_t)cus * 4 * 8 * 8));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  run_all<0>(cus, d, dc, e0, e1, ghz);
  CHK(hipDeviceSynchronize());
  CHK(hipFree(d));
  CHK(hipFree(dc));
  return 0;
}
