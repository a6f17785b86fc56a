// Integer / f64 VALU issue-rate microbenchmark for gfx950 (MI355X).
// Each lane runs ITERS iterations of 8 independent chains of ONE instruction
// (inline asm so the compiler cannot substitute another opcode).  Rate is
// reported as lane-ops/s and as a fraction of the full-rate VALU ceiling
// (256 CU x 4 SIMD x 32 lanes x clock).  Used to pick the GF(2^255-19) limb
// schedule (DESIGN.md "field arithmetic").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_mad64(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  uint32_t x = a + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c) : "v"(x), "v"(b) : "vcc");
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_mullo(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(c) : "v"(b));
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_mulhi(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(c) : "v"(b));
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_addc(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(c) : "v"(b) : "vcc");
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_add(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(c) : "v"(b));
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_mad24(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  uint32_t x = a + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(c) : "v"(x), "v"(b));
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_fma64(uint64_t* out, uint32_t a, uint32_t b) {
  double c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  double x = 1.0000001 + a, y = 0.999999 * b;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(c) : "v"(x), "v"(y));
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  double r = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = __double_as_longlong(r);
}

__global__ void k_lshr64(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(c));
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_alignbit(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define M(c) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(c) : "v"(b));
    M(c0) M(c1) M(c2) M(c3) M(c4) M(c5) M(c6) M(c7)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

typedef void (*kfn)(uint64_t*, uint32_t, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  double clk = prop.clockRate * 1e3;
  printf("device %s CUs=%d clock=%.0f MHz\n", prop.gcnArchName, cus, clk / 1e6);
  const int block = 256;
  const int grid = cus * 8;  // 8 waves/SIMD-quad... 8 blocks x 4 waves = 32 waves/CU
  uint64_t* d;
  CHK(hipMalloc(&d, sizeof(uint64_t) * grid * block));
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
    {"v_addc_co_u32", k_addc}, {"v_add_u32", k_add}, {"v_mad_u32_u24", k_mad24},
    {"v_fma_f64", k_fma64}, {"v_lshrrev_b64", k_lshr64}, {"v_alignbit_b32", k_alignbit}};
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, d, 3u, 5u);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      double ops = (double)grid * block * ITERS * 8;
      double rate = ops / (ms * 1e-3);
      double peak = (double)cus * 4 * 32 * clk;
      if (rep == 2) printf("%-16s %8.3f ms  %.3e lane-op/s  = %.3f of full-rate VALU (%.3e)\n", k.name, ms, rate, rate / peak, peak);
    }
  }
  CHK(hipFree(d));
  return 0;
}
