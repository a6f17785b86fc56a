// Per-SIMD issue cost of the integer instructions the GF(2^255-19) code is
// made of, on gfx950 (MI355X), measured in shader cycles with s_memtime so the
// result does not depend on the clock the chip holds under load.
//
//   * "thru W=w": 16 independent chains of one instruction per lane, w waves
//     on each SIMD (one workgroup of 256*w threads per CU, forced by LDS);
//     reported as SIMD cycles per wave-instruction.
//   * "lat": one dependent chain, one wave per SIMD: cycles per instruction.
//   * fe_mul / fe_sq of stl_fe25519.h in two independent chains per lane, at
//     1..4 waves per SIMD: SIMD cycles per wave-level field operation.
//
// Used to choose the reduction schedule of the field multiply.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#include "../../stellard_amd/csrc/stl_fe25519.h"

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define ITERS 512

// ---- single-instruction kernels ----
#define BODY16(M) M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7) M(c8) M(c9) M(c10) M(c11) M(c12) M(c13) M(c14) M(c15)
#define DECL64 uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, \
  c7 = c0 + 7, c8 = c0 + 8, c9 = c0 + 9, c10 = c0 + 10, c11 = c0 + 11, c12 = c0 + 12, c13 = c0 + 13, c14 = c0 + 14, c15 = c0 + 15;
#define DECL32 uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, \
  c7 = c0 + 7, c8 = c0 + 8, c9 = c0 + 9, c10 = c0 + 10, c11 = c0 + 11, c12 = c0 + 12, c13 = c0 + 13, c14 = c0 + 14, c15 = c0 + 15;
#define FOLD (c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7 ^ c8 ^ c9 ^ c10 ^ c11 ^ c12 ^ c13 ^ c14 ^ c15)

#define KERNEL(NAME, DECL, ASM, ...)                                                   \
  __global__ void NAME(uint64_t* out, uint64_t* cyc, uint32_t a, uint32_t b) {        \
    DECL uint32_t x = a + threadIdx.x;                                                \
    (void)x;                                                                          \
    __syncthreads();                                                                  \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                 \
    for (int i = 0; i < ITERS; ++i) {                                                 \
      _Pragma("unroll 1") for (int r = 0; r < 1; ++r) {                               \
        BODY16(ASM)                                                                   \
      }                                                                               \
    }                                                                                 \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                 \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)FOLD;                      \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
  }

#define A_MAD64(c) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c) : "v"(x), "v"(b) : "vcc");
#define A_LSHR64(c) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(c));
#define A_LSHLADD64(c) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(c));
#define A_ADD(c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(c) : "v"(b));
#define A_AND(c) asm volatile("v_and_b32 %0, %0, %1" : "+v"(c) : "v"(b));
#define A_ALIGN(c) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(c) : "v"(b));
#define A_MAD24(c) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(c) : "v"(x), "v"(b));
#define A_MULHI24(c) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(c) : "v"(b));
#define A_MULLO(c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(c) : "v"(b));
#define A_MULHI(c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(c) : "v"(b));
#define A_CND(c) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(c) : "v"(b) : "vcc");
#define A_ADD3(c) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(c) : "v"(b));
#define A_BFE(c) asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(c));
#define A_ADDCO(c) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(c) : "v"(b) : "vcc");
#define A_DOT2(c) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(c) : "v"(x), "v"(b));
#define A_ANDLIT(c) asm volatile("v_and_b32_e32 %0, 0x1fffffff, %0" : "+v"(c));
#define A_ANDSG(c) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(c) : "s"(b));
#define A_ADDE64(c) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(c) : "v"(b));
#define A_MAD64S(c) { uint64_t cc_; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c), "=s"(cc_) : "v"(x), "v"(b)); }

KERNEL(k_mad64, DECL64, A_MAD64)
KERNEL(k_lshr64, DECL64, A_LSHR64)
KERNEL(k_lshladd64, DECL64, A_LSHLADD64)
KERNEL(k_add, DECL32, A_ADD)
KERNEL(k_and, DECL32, A_AND)
KERNEL(k_align, DECL32, A_ALIGN)
KERNEL(k_mad24, DECL32, A_MAD24)
KERNEL(k_mulhi24, DECL32, A_MULHI24)
KERNEL(k_mullo, DECL32, A_MULLO)
KERNEL(k_mulhi, DECL32, A_MULHI)
KERNEL(k_cnd, DECL32, A_CND)
KERNEL(k_add3, DECL32, A_ADD3)
KERNEL(k_bfe, DECL32, A_BFE)
KERNEL(k_addco, DECL32, A_ADDCO)
KERNEL(k_dot2, DECL32, A_DOT2)
KERNEL(k_andlit, DECL32, A_ANDLIT)
KERNEL(k_andsg, DECL32, A_ANDSG)
KERNEL(k_adde64, DECL32, A_ADDE64)
KERNEL(k_mad64s, DECL64, A_MAD64S)
// 8 mad64 chains interleaved with 8 literal-and chains (the fe_mul mix)
__global__ void k_mix(uint64_t* out, uint64_t* cyc, uint32_t a, uint32_t b) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  uint32_t d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
  uint32_t x = a + threadIdx.x;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
#define P(c, d) A_MAD64S(c) A_ANDLIT(d)
    P(c0, d0) P(c1, d1) P(c2, d2) P(c3, d3) P(c4, d4) P(c5, d5) P(c6, d6) P(c7, d7)
#undef P
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7 ^ d0 ^ d1 ^ d2 ^ d3 ^ d4 ^ d5 ^ d6 ^ d7;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

// dependent-chain latency: one chain per lane
#define LATK(NAME, T, ASM1)                                                           \
  __global__ void NAME(uint64_t* out, uint64_t* cyc, uint32_t a, uint32_t b) {        \
    T c = threadIdx.x; uint32_t x = a + threadIdx.x; (void)x;                         \
    __syncthreads();                                                                  \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                 \
    for (int i = 0; i < ITERS; ++i) { ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) \
                                      ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) ASM1(c) } \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                 \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)c;                         \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
  }
LATK(l_mad64, uint64_t, A_MAD64)
LATK(l_lshr64, uint64_t, A_LSHR64)
LATK(l_lshladd64, uint64_t, A_LSHLADD64)
LATK(l_add, uint32_t, A_ADD)

// ---- manual two-way interleave of independent field multiplies: each mad is
// ordered by an empty asm on its accumulator, so the column chains start from
// their carry-in (no reassociation) and the ILP comes from the partner product.
#define MADF(acc, x, y)                     \
  do {                                      \
    acc += (uint64_t)(x) * (y);             \
    asm volatile("" : "+v"(acc));           \
  } while (0)

__device__ __forceinline__ void fe_mul2_manual(stl::fe& h1, const stl::fe& a1, const stl::fe& b1, stl::fe& h2,
                                               const stl::fe& a2, const stl::fe& b2) {
  const stl::fe A1 = a1, B1 = b1, A2 = a2, B2 = b2;
  uint64_t hc1[8], hc2[8];
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    uint64_t c1 = 0, c2 = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      MADF(c1, A1.v[i], B1.v[j]);
      MADF(c2, A2.v[i], B2.v[j]);
    }
    hc1[k - 9] = c1;
    hc2[k - 9] = c2;
  }
  uint64_t cy1 = 0, cy2 = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    uint64_t c1 = cy1, c2 = cy2;
    if (k < 8) {
      MADF(c1, (uint32_t)hc1[k], 1216u);
      MADF(c2, (uint32_t)hc2[k], 1216u);
    }
    if (k > 0) {
      MADF(c1, (uint32_t)(hc1[k - 1] >> 32), 9728u);
      MADF(c2, (uint32_t)(hc2[k - 1] >> 32), 9728u);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      MADF(c1, A1.v[i], B1.v[j]);
      MADF(c2, A2.v[i], B2.v[j]);
    }
    h1.v[k] = (uint32_t)c1 & stl::M29;
    h2.v[k] = (uint32_t)c2 & stl::M29;
    cy1 = c1 >> 29;
    cy2 = c2 >> 29;
  }
  uint64_t u1 = (uint64_t)h1.v[0] + cy1 * 1216u, u2 = (uint64_t)h2.v[0] + cy2 * 1216u;
  h1.v[0] = (uint32_t)u1 & stl::M29;
  h1.v[1] += (uint32_t)(u1 >> 29);
  h2.v[0] = (uint32_t)u2 & stl::M29;
  h2.v[1] += (uint32_t)(u2 >> 29);
}

// ---- field-operation kernels: two independent chains per lane ----
#define FE_ITERS 64
template <int OP>
__global__ void k_fe(uint64_t* out, uint64_t* cyc, uint32_t a0, uint32_t b0) {
  stl::fe a, b, c, d;
  for (int i = 0; i < 9; ++i) {
    a.v[i] = (threadIdx.x * 2654435761u + i * a0) & stl::M29;
    b.v[i] = (0x9e3779b9u * (i + b0) + threadIdx.x * 77u) & stl::M29;
    c.v[i] = a.v[i] ^ 0x55u;
    d.v[i] = b.v[i] ^ 0x1234u;
  }
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < FE_ITERS; ++i) {
    if (OP == 0) { stl::fe_mul(a, a, b); stl::fe_mul(c, c, d); }
    if (OP == 1) { stl::fe_sq(a, a); stl::fe_sq(c, c); }
    if (OP == 2) { stl::fe_sub(a, a, b); stl::fe_sub(c, c, d); }
    if (OP == 3) { fe_mul2_manual(a, a, b, c, c, d); }
    if (OP == 4) { stl::fe_mul2(a, a, b, c, c, d); }
    if (OP == 5) { stl::fe_mul(a, a, b); stl::fe_mul(c, c, d); }
    if (OP == 6) { stl::fe_sq2(a, a, c, c); }
    if (OP == 7) { stl::fe_sq(a, a); stl::fe_sq(c, c); }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= a.v[i] ^ c.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

typedef void (*kfn)(uint64_t*, uint64_t*, uint32_t, uint32_t);

// cycles per wave-instruction on one SIMD, w waves per SIMD
static int run(kfn f, int cus, int w, double instrs_per_wave, double* out_simd_cycles, uint64_t* d, uint64_t* dc) {
  const int wgs = w > 4 ? w / 4 : 1;              // workgroups per CU
  const int block = 256 * w / wgs;
  const int lds = wgs == 1 ? 96 * 1024 : 64 * 1024; // forces wgs workgroups per CU
  CHK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  std::vector<uint64_t> cyc(cus * wgs * block / 64);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(f, dim3(cus * wgs), dim3(block), lds, 0, d, dc, 3u, 5u);
    CHK(hipDeviceSynchronize());
  }
  CHK(hipMemcpy(cyc.data(), dc, cyc.size() * 8, hipMemcpyDeviceToHost));
  std::sort(cyc.begin(), cyc.end());
  // waves sharing a SIMD finish at different times (issue priority by age):
  // the SIMD is busy until its last wave ends, so cost = max wave cycles / (w * instrs)
  const double mx = (double)cyc.back();
  *out_simd_cycles = mx / (w * instrs_per_wave);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs=%d\n", prop.gcnArchName, cus);
  uint64_t *d, *dc;
  CHK(hipMalloc(&d, sizeof(uint64_t) * cus * 2048));
  CHK(hipMalloc(&dc, sizeof(uint64_t) * cus * 32));
  struct { const char* name; kfn f; } ks[] = {
      {"v_mad_u64_u32", k_mad64}, {"v_lshrrev_b64", k_lshr64}, {"v_lshl_add_u64", k_lshladd64},
      {"v_add_u32", k_add}, {"v_and_b32", k_and}, {"v_alignbit_b32", k_align}, {"v_mad_u32_u24", k_mad24},
      {"v_mul_hi_u32_u24", k_mulhi24}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
      {"v_cndmask_b32", k_cnd}, {"v_add3_u32", k_add3}, {"v_bfe_u32", k_bfe}, {"v_add_co_u32", k_addco},
      {"v_dot2_u32_u16", k_dot2}, {"v_and_b32 literal", k_andlit}, {"v_and_b32 sgpr", k_andsg},
      {"v_add_u32_e64", k_adde64}, {"v_mad_u64_u32 sgpr", k_mad64s}, {"mad64+and pair", k_mix}};
  printf("%-18s %10s %10s %10s %10s\n", "instruction", "W=1", "W=2", "W=4", "W=8");
  for (auto& k : ks) {
    double c1, c2, c4, c8;
    if (run(k.f, cus, 1, ITERS * 16.0, &c1, d, dc) || run(k.f, cus, 2, ITERS * 16.0, &c2, d, dc) ||
        run(k.f, cus, 4, ITERS * 16.0, &c4, d, dc) || run(k.f, cus, 8, ITERS * 16.0, &c8, d, dc))
      return 1;
    printf("%-18s %10.2f %10.2f %10.2f %10.2f   (SIMD cycles / wave-instr)\n", k.name, c1, c2, c4, c8);
  }
  struct { const char* name; kfn f; } ls[] = {
      {"v_mad_u64_u32", l_mad64}, {"v_lshrrev_b64", l_lshr64}, {"v_lshl_add_u64", l_lshladd64}, {"v_add_u32", l_add}};
  for (auto& k : ls) {
    double c1;
    if (run(k.f, cus, 1, ITERS * 16.0, &c1, d, dc)) return 1;
    printf("latency %-18s %8.2f cycles (dependent chain, 1 wave/SIMD)\n", k.name, c1);
  }
  struct { const char* name; kfn f; } fs[] = {{"fe_mul", k_fe<0>}, {"fe_sq", k_fe<1>}, {"fe_sub", k_fe<2>}, {"fe_mul2", k_fe<3>}, {"mul2_n", k_fe<4>}, {"mul1_n", k_fe<5>},
                                        {"sq2_n", k_fe<6>}, {"sq1_n", k_fe<7>}};
  for (auto& k : fs) {
    printf("%-8s", k.name);
    for (int w = 1; w <= 4; ++w) {
      double c;
      if (run(k.f, cus, w, FE_ITERS * 2.0, &c, d, dc)) return 1;
      printf("  W=%d %7.1f", w, c);
    }
    printf("   (SIMD cycles / wave-op)\n");
  }
  return 0;
}
