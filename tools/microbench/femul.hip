// GF(2^255-19) multiply throughput for candidate limb schedules on gfx950.
// Decides the field representation of the verify kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define ITERS 256

struct fe8 { uint32_t v[8]; };
struct fe9 { uint32_t v[9]; };

// ---- variant A: 8x32 saturated, inline-asm mac with SGPR carry ----
__device__ __forceinline__ void macA(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(hi) : "v"(a), "v"(b));
}
__device__ __forceinline__ void macA0(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, 0, %1"
      : "+v"(acc), "=&s"(cc), "=v"(hi) : "v"(a), "v"(b));
}
// ---- variant B: same with VCC ----
__device__ __forceinline__ void macB(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(hi) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ void macB0(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_cndmask_b32_e64 %1, 0, 1, vcc"
      : "+v"(acc), "=v"(hi) : "v"(a), "v"(b) : "vcc");
}

template <int V>
__device__ __forceinline__ void mul8(fe8& r, const fe8& a, const fe8& b) {
  uint32_t t[16];
  uint64_t acc = 0; uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) {
    bool first = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int j = k - i;
      if (j < 0 || j > 7) continue;
      if (V == 0) { if (first) macA0(acc, hi, a.v[i], b.v[j]); else macA(acc, hi, a.v[i], b.v[j]); }
      else { if (first) macB0(acc, hi, a.v[i], b.v[j]); else macB(acc, hi, a.v[i], b.v[j]); }
      first = false;
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
  }
  t[15] = (uint32_t)acc;
  uint32_t u[8]; uint64_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) { m = (uint64_t)t[8 + i] * 38u + (m >> 32); u[i] = (uint32_t)m; }
  uint32_t top = (uint32_t)(m >> 32);
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) { s = (uint64_t)t[i] + u[i] + (s >> 32); r.v[i] = (uint32_t)s; }
  top += (uint32_t)(s >> 32);
  s = (uint64_t)top * 38u;
#pragma unroll
  for (int i = 0; i < 8; ++i) { s = (uint64_t)r.v[i] + s; r.v[i] = (uint32_t)s; s >>= 32; }
  r.v[0] += (uint32_t)s * 38u;
}

// ---- variant C: 8x32 with unsigned __int128 accumulator ----
__device__ __forceinline__ void mul8c(fe8& r, const fe8& a, const fe8& b) {
  uint32_t t[16];
  unsigned __int128 acc = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int j = k - i;
      if (j < 0 || j > 7) continue;
      acc += (uint64_t)a.v[i] * b.v[j];
    }
    t[k] = (uint32_t)acc;
    acc >>= 32;
  }
  t[15] = (uint32_t)acc;
  uint32_t u[8]; uint64_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) { m = (uint64_t)t[8 + i] * 38u + (m >> 32); u[i] = (uint32_t)m; }
  uint32_t top = (uint32_t)(m >> 32);
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) { s = (uint64_t)t[i] + u[i] + (s >> 32); r.v[i] = (uint32_t)s; }
  top += (uint32_t)(s >> 32);
  s = (uint64_t)top * 38u;
#pragma unroll
  for (int i = 0; i < 8; ++i) { s = (uint64_t)r.v[i] + s; r.v[i] = (uint32_t)s; s >>= 32; }
  r.v[0] += (uint32_t)s * 38u;
}

// ---- variant D: 9 x 29-bit unsaturated limbs, pure mad64 columns ----
#define M29 0x1fffffffu
__device__ __forceinline__ void mul9(fe9& r, const fe9& a, const fe9& b) {
  uint64_t c[18];
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      int j = k - i;
      if (j < 0 || j > 8) continue;
      acc += (uint64_t)a.v[i] * b.v[j];
    }
    c[k] = acc;
  }
  // normalize high columns 9..16 into 29-bit digits, carry to c[17]
  uint64_t carry = 0;
#pragma unroll
  for (int k = 9; k < 17; ++k) { uint64_t t = c[k] + carry; c[k] = t & M29; carry = t >> 29; }
  c[17] = carry;
  // fold: 2^261 = 2^6 * 2^255 == 64*19 = 1216
#pragma unroll
  for (int k = 9; k < 18; ++k) c[k - 9] += c[k] * 1216u;
  carry = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) { uint64_t t = c[k] + carry; r.v[k] = (uint32_t)t & M29; carry = t >> 29; }
  // carry has weight 2^261
  uint64_t t = (uint64_t)r.v[0] + carry * 1216u;
  r.v[0] = (uint32_t)t & M29;
  r.v[1] += (uint32_t)(t >> 29);
}

template <int V>
__global__ __launch_bounds__(256) void k8(fe8* p, int n) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fe8 a, b, a2;
#pragma unroll
  for (int i = 0; i < 8; ++i) { a.v[i] = tid * 2654435761u + i; b.v[i] = 0x9e3779b9u * (i + 1); a2.v[i] = a.v[i] ^ 0x55; }
  for (int i = 0; i < n; ++i) {
    if (V == 2) { mul8c(a, a, b); mul8c(a2, a2, b); }
    else { mul8<V>(a, a, b); mul8<V>(a2, a2, b); }
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= a.v[i] ^ a2.v[i];
  p[tid].v[0] = x;
}

__global__ __launch_bounds__(256) void k9(fe8* p, int n) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fe9 a, b, a2;
#pragma unroll
  for (int i = 0; i < 9; ++i) { a.v[i] = (tid * 2654435761u + i) & M29; b.v[i] = (0x9e3779b9u * (i + 1)) & M29; a2.v[i] = a.v[i] ^ 0x55; }
  for (int i = 0; i < n; ++i) { mul9(a, a, b); mul9(a2, a2, b); }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) x ^= a.v[i] ^ a2.v[i];
  p[tid].v[0] = x;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  const int block = 256, grid = cus * 8;
  fe8* d;
  CHK(hipMalloc(&d, sizeof(fe8) * grid * block));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  struct { const char* name; void (*f)(fe8*, int); } ks[] = {
      {"A: 8x32 asm mac (sgpr carry)", k8<0>}, {"B: 8x32 asm mac (vcc)", k8<1>},
      {"C: 8x32 __int128 accum", k8<2>}, {"D: 9x29 unsaturated", k9}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, d, ITERS);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      double muls = 2.0 * grid * block * ITERS;
      if (rep == 2) printf("%-32s %8.3f ms  %.3e fe_mul/s  (%.1f ns/mul/lane-equiv)\n", k.name, ms, muls / (ms * 1e-3), 1e9 * ms * 1e-3 / muls);
    }
  }
  return 0;
}
