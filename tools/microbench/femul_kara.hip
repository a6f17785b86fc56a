// femul_kara.hip -- does a one-level 3x3 Karatsuba split of the 9x29-bit
// product pay on gfx950?  
//
// Three product implementations, each run as two independent dependent chains
// per lane (the shape of fe_mul2 in the verify kernels), same fold-by-halves
// reduction, same limb bounds:
//   prod   stl::fe_mul2 from stl_fe25519.h -- the production, hand-scheduled
//          schoolbook (81 + 17 fold mads per product);
//   school compiler-scheduled schoolbook with the same fold (reference point);
//   kara   a = A0 + A1 X + A2 X^2 (X = 2^87, three limbs each): 6 products
//          of 3x3 limbs (54 mads) + 18 limb pre-adds + the recombination
//          (Q01-P00-P11, Q02-P00-P22+P11, Q12-P11-P22 on 64-bit columns),
//          then the same fold.
// Prints products/s per variant and checks all three agree bit for bit.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I stellard_amd/csrc tools/microbench/femul_kara.hip -o femul_kara
#include <hip/hip_runtime.h>

#include <cstdio>

#include "stl_fe25519.h"

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                 \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

using stl::fe;
constexpr uint32_t M29 = 0x1fffffffu;

// reduce 17 raw 64-bit columns (fold by halves, as fe_prod_n) into h
__device__ __forceinline__ void reduce17(fe& h, const uint64_t c[17]) {
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    uint64_t acc = c[k] + carry;
    if (k < 8) acc += (uint64_t)(uint32_t)c[k + 9] * 1216u;
    if (k > 0) acc += (uint64_t)(uint32_t)(c[k + 8] >> 32) * 9728u;
    h.v[k] = (uint32_t)acc & M29;
    carry = acc >> 29;
  }
  const uint64_t u = (uint64_t)h.v[0] + carry * 1216u;
  h.v[0] = (uint32_t)u & M29;
  h.v[1] += (uint32_t)(u >> 29);
}

__device__ __forceinline__ void school(fe& h, const fe& a, const fe& b) {
  uint64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 9) acc += (uint64_t)a.v[i] * b.v[j];
    }
    c[k] = acc;
  }
  reduce17(h, c);
}

// 3x3 limb polynomial product: 5 columns
__device__ __forceinline__ void p33(uint64_t o[5], const uint32_t* x, const uint32_t* y) {
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 3) acc += (uint64_t)x[i] * y[j];
    }
    o[k] = acc;
  }
}

__device__ __forceinline__ void kara(fe& h, const fe& a, const fe& b) {
  uint32_t s01a[3], s02a[3], s12a[3], s01b[3], s02b[3], s12b[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    s01a[i] = a.v[i] + a.v[3 + i];
    s02a[i] = a.v[i] + a.v[6 + i];
    s12a[i] = a.v[3 + i] + a.v[6 + i];
    s01b[i] = b.v[i] + b.v[3 + i];
    s02b[i] = b.v[i] + b.v[6 + i];
    s12b[i] = b.v[3 + i] + b.v[6 + i];
  }
  uint64_t P00[5], P11[5], P22[5], Q01[5], Q02[5], Q12[5];
  p33(P00, &a.v[0], &b.v[0]);
  p33(P11, &a.v[3], &b.v[3]);
  p33(P22, &a.v[6], &b.v[6]);
  p33(Q01, s01a, s01b);
  p33(Q02, s02a, s02b);
  p33(Q12, s12a, s12b);
  uint64_t c[17];
#pragma unroll
  for (int t = 0; t < 17; ++t) c[t] = 0;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    c[u] += P00[u];
    c[3 + u] += Q01[u] - P00[u] - P11[u];
    c[6 + u] += Q02[u] - P00[u] - P22[u] + P11[u];
    c[9 + u] += Q12[u] - P11[u] - P22[u];
    c[12 + u] += P22[u];
  }
  reduce17(h, c);
}

template <int V>
__global__ __launch_bounds__(256) void kbench(uint32_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b, a2;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    a.v[i] = (tid * 2654435761u + 977u * i) & M29;
    b.v[i] = (0x9e3779b9u * (i + 1)) & M29;
    a2.v[i] = a.v[i] ^ 0x55u;
  }
  for (int i = 0; i < iters; ++i) {
    if (V == 0) {
      stl::fe_mul2(a, a, b, a2, a2, b);
    } else if (V == 1) {
      school(a, a, b);
      school(a2, a2, b);
    } else {
      kara(a, a, b);
      kara(a2, a2, b);
    }
  }
  uint32_t w[8], w2[8];
  stl::fe_tobytes(w, a);
  stl::fe_tobytes(w2, a2);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[(size_t)tid * 16 + i] = w[i], out[(size_t)tid * 16 + 8 + i] = w2[i];
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int block = 256, iters = 512;
  const char* names[3] = {"prod (stl::fe_mul2, hand-scheduled)", "school (compiler-scheduled)",
                          "kara (3x3 Karatsuba)"};
  void (*ks[3])(uint32_t*, int) = {kbench<0>, kbench<1>, kbench<2>};
  for (int waves = 2; waves <= 4; waves += 2) {
    const int grid = prop.multiProcessorCount * 4 * waves / 4;  // 4 waves per block -> `waves` waves per SIMD
    uint32_t* d[3];
    for (int v = 0; v < 3; ++v) CHK(hipMalloc(&d[v], sizeof(uint32_t) * 16 * (size_t)grid * block));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int v = 0; v < 3; ++v) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(ks[v], dim3(grid), dim3(block), 0, 0, d[v], iters);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      const double prods = 2.0 * grid * block * iters;
      printf("waves/SIMD %d  %-38s %8.3f ms  %.3e products/s\n", waves, names[v], best, prods / (best * 1e-3));
    }
    // parity: the three variants produce the same field elements
    const size_t words = (size_t)16 * grid * block;
    uint32_t* h[3];
    int bad = 0;
    for (int v = 0; v < 3; ++v) {
      h[v] = new uint32_t[words];
      CHK(hipMemcpy(h[v], d[v], words * 4, hipMemcpyDeviceToHost));
    }
    for (size_t i = 0; i < words; ++i) bad += (h[0][i] != h[1][i]) + (h[0][i] != h[2][i]);
    printf("waves/SIMD %d  parity: %s (%d differing words)\n", waves, bad ? "MISMATCH" : "all equal", bad);
    for (int v = 0; v < 3; ++v) {
      delete[] h[v];
      CHK(hipFree(d[v]));
    }
    if (bad) return 2;
  }
  return 0;
}
