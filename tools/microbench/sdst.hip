// Does a VALU instruction's SGPR carry-out serialize a wave's issue?
// v_mad_u64_u32 (and v_add_co_u32) write a carry-out SGPR pair; the compiler
// gives every mad of a field product the same (dead) pair.  A single wave
// issued a mad64 only every ~9.2 SIMD cycles in isarate.hip, against ~5 for
// 64-bit ops without an SGPR result (v_lshl_add_u64).  Here the carry-out goes
// to the same pair (vcc, or s[20:21]) or to 2 / 4 / 8 rotating pairs, 16
// independent chains per lane, 1 / 2 / 4 waves per SIMD, SIMD cycles per
// wave-instruction (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define ITERS 512

#define MAD_SD(c, sd) asm volatile("v_mad_u64_u32 %0, " sd ", %1, %2, %0" : "+v"(c) : "v"(x), "v"(b) : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s36", "s37", "s38", "s39", "vcc");
#define ADDCO_SD(c, sd) asm volatile("v_add_co_u32 %0, " sd ", %0, %1" : "+v"(c) : "v"(b) : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s36", "s37", "s38", "s39", "vcc");
#define LSHLADD(c) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(c));

#define S1 "s[20:21]"
#define P0 "s[20:21]"
#define P1 "s[22:23]"
#define P2 "s[24:25]"
#define P3 "s[26:27]"
#define P4 "s[28:29]"
#define P5 "s[30:31]"
#define P6 "s[36:37]"
#define P7 "s[38:39]"

#define DECL64 uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, \
  c7 = c0 + 7, c8 = c0 + 8, c9 = c0 + 9, c10 = c0 + 10, c11 = c0 + 11, c12 = c0 + 12, c13 = c0 + 13, c14 = c0 + 14, c15 = c0 + 15;
#define DECL32 uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, \
  c7 = c0 + 7, c8 = c0 + 8, c9 = c0 + 9, c10 = c0 + 10, c11 = c0 + 11, c12 = c0 + 12, c13 = c0 + 13, c14 = c0 + 14, c15 = c0 + 15;
#define FOLD (c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7 ^ c8 ^ c9 ^ c10 ^ c11 ^ c12 ^ c13 ^ c14 ^ c15)

#define KERNEL(NAME, DECL, BODY)                                                      \
  __global__ void NAME(uint64_t* out, uint64_t* cyc, uint32_t a, uint32_t b) {        \
    DECL uint32_t x = a + threadIdx.x;                                                \
    (void)x;                                                                          \
    __syncthreads();                                                                  \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                 \
    for (int i = 0; i < ITERS; ++i) { BODY }                                          \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                 \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)FOLD;                      \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
  }

#define M16(OP, A, B, C, D, E, F, G, H) OP(c0, A) OP(c1, B) OP(c2, C) OP(c3, D) OP(c4, E) OP(c5, F) OP(c6, G) OP(c7, H) \
  OP(c8, A) OP(c9, B) OP(c10, C) OP(c11, D) OP(c12, E) OP(c13, F) OP(c14, G) OP(c15, H)

KERNEL(k_mad_vcc, DECL64, M16(MAD_SD, "vcc", "vcc", "vcc", "vcc", "vcc", "vcc", "vcc", "vcc"))
KERNEL(k_mad_s1, DECL64, M16(MAD_SD, S1, S1, S1, S1, S1, S1, S1, S1))
KERNEL(k_mad_s2, DECL64, M16(MAD_SD, P0, P1, P0, P1, P0, P1, P0, P1))
KERNEL(k_mad_s4, DECL64, M16(MAD_SD, P0, P1, P2, P3, P0, P1, P2, P3))
KERNEL(k_mad_s8, DECL64, M16(MAD_SD, P0, P1, P2, P3, P4, P5, P6, P7))
KERNEL(k_addco_vcc, DECL32, M16(ADDCO_SD, "vcc", "vcc", "vcc", "vcc", "vcc", "vcc", "vcc", "vcc"))
KERNEL(k_addco_s8, DECL32, M16(ADDCO_SD, P0, P1, P2, P3, P4, P5, P6, P7))
#define LSHLADD_(c, s) LSHLADD(c)
KERNEL(k_lshladd, DECL64, M16(LSHLADD_, 0, 0, 0, 0, 0, 0, 0, 0))


// The same without clobber lists: the compiler sees no SGPR write, so it puts
// no hazard s_nop between the mads (the clobbering forms above get one after
// every mad, which a lone wave pays as a full issue slot).
#define MAD_NC(c, sd) asm volatile("v_mad_u64_u32 %0, " sd ", %1, %2, %0" : "+v"(c) : "v"(x), "v"(b));
#define Q0 "s[40:41]"
#define Q1 "s[42:43]"
#define Q2 "s[44:45]"
#define Q3 "s[46:47]"
#define Q4 "s[48:49]"
#define Q5 "s[50:51]"
#define Q6 "s[52:53]"
#define Q7 "s[54:55]"
KERNEL(k_madnc_one, DECL64, M16(MAD_NC, Q0, Q0, Q0, Q0, Q0, Q0, Q0, Q0))
KERNEL(k_madnc_s2, DECL64, M16(MAD_NC, Q0, Q1, Q0, Q1, Q0, Q1, Q0, Q1))
KERNEL(k_madnc_s4, DECL64, M16(MAD_NC, Q0, Q1, Q2, Q3, Q0, Q1, Q2, Q3))
KERNEL(k_madnc_s8, DECL64, M16(MAD_NC, Q0, Q1, Q2, Q3, Q4, Q5, Q6, Q7))

typedef void (*kfn)(uint64_t*, uint64_t*, uint32_t, uint32_t);

static int run(kfn f, int cus, int w, double instrs_per_wave, double* out_simd_cycles, uint64_t* d, uint64_t* dc) {
  const int wgs = w > 4 ? w / 4 : 1;
  const int block = 256 * w / wgs;
  const int lds = wgs == 1 ? 96 * 1024 : 64 * 1024;
  CHK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  std::vector<uint64_t> cyc(cus * wgs * block / 64);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(f, dim3(cus * wgs), dim3(block), lds, 0, d, dc, 3u, 5u);
    CHK(hipDeviceSynchronize());
  }
  CHK(hipMemcpy(cyc.data(), dc, cyc.size() * 8, hipMemcpyDeviceToHost));
  std::sort(cyc.begin(), cyc.end());
  *out_simd_cycles = (double)cyc.back() / (w * instrs_per_wave);
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
      {"mad64 sdst vcc", k_mad_vcc}, {"mad64 sdst one pair", k_mad_s1}, {"mad64 sdst 2 pairs", k_mad_s2},
      {"mad64 sdst 4 pairs", k_mad_s4}, {"mad64 sdst 8 pairs", k_mad_s8}, {"add_co vcc", k_addco_vcc},
      {"add_co 8 pairs", k_addco_s8}, {"v_lshl_add_u64", k_lshladd},
      {"mad64 no-nop one pair", k_madnc_one}, {"mad64 no-nop 2 pairs", k_madnc_s2},
      {"mad64 no-nop 4 pairs", k_madnc_s4}, {"mad64 no-nop 8 pairs", k_madnc_s8}};
  printf("%-22s %10s %10s %10s\n", "instruction", "W=1", "W=2", "W=4");
  for (auto& k : ks) {
    double c1, c2, c4;
    if (run(k.f, cus, 1, ITERS * 16.0, &c1, d, dc) || run(k.f, cus, 2, ITERS * 16.0, &c2, d, dc) ||
        run(k.f, cus, 4, ITERS * 16.0, &c4, d, dc))
      return 1;
    printf("%-22s %10.2f %10.2f %10.2f   (SIMD cycles / wave-instr)\n", k.name, c1, c2, c4);
  }
  return 0;
}
