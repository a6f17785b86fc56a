// Main-loop occupancy experiment: SIMD cycles per double_scalarmult
// ([k](-A) + [S]B, the verify kernel's Straus loop, stl_verify_core.h) at
// W = 2, 3, 4 waves per SIMD, timed in shader cycles with s_memtime.
// Field values are arbitrary (the loop's cost does not depend on them).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#include "../../stellard_amd/csrc/stl_base_table.h"
#include "../../stellard_amd/csrc/stl_verify_core.h"

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int W>
__global__ __launch_bounds__(256, W) void k_smul(uint4* ws, uint32_t* out, uint64_t* cyc) {
  __shared__ uint32_t sB[stl::kBaseTableEntries * stl::kBaseNielsWords];
  for (uint32_t i = threadIdx.x; i < (uint32_t)(stl::kBaseTableEntries * stl::kBaseNielsWords); i += 256)
    sB[i] = (&stl::kBaseNiels[0][0])[i];
  __syncthreads();
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
  stl::TableView tv{ws + (size_t)gid * 81, 1};
  uint32_t k[8], S[8];
  uint32_t h = gid * 2654435761u + 12345u;
  for (int i = 0; i < 8; ++i) { h ^= h << 13; h ^= h >> 17; h ^= h << 5; k[i] = h; h ^= h << 13; h ^= h >> 17; h ^= h << 5; S[i] = h; }
  k[7] &= 0x0fffffffu; S[7] &= 0x0fffffffu;
  stl::ge_p3 negA;
  for (int i = 0; i < 9; ++i) {
    negA.X.v[i] = (h * (i + 1)) & stl::M29; negA.Y.v[i] = (h * (i + 7)) & stl::M29;
    negA.Z.v[i] = (h * (i + 3)) & stl::M29; negA.T.v[i] = (h * (i + 5)) & stl::M29;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  stl::ge_p2 r;
  stl::double_scalarmult(r, negA, k, S, tv, sB);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= r.X.v[i] ^ r.Y.v[i] ^ r.Z.v[i];
  out[gid] = x;
  if ((threadIdx.x & 63) == 0) cyc[gid / 64] = t1 - t0;
}

template <int W>
static int run(int cus, uint4* ws, uint32_t* out, uint64_t* dc) {
  const int grid = cus * W;
  std::vector<uint64_t> cyc(grid * 4);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_smul<W>, dim3(grid), dim3(256), 0, 0, ws, out, dc);
    CHK(hipDeviceSynchronize());
  }
  CHK(hipMemcpy(cyc.data(), dc, cyc.size() * 8, hipMemcpyDeviceToHost));
  std::sort(cyc.begin(), cyc.end());
  const double med = (double)cyc[cyc.size() / 2];
  printf("W=%d  wave cycles %.0f (min %llu max %llu)  SIMD cycles per scalarmult %.0f (max/W)\n", W, med,
         (unsigned long long)cyc.front(), (unsigned long long)cyc.back(), (double)cyc.back() / W);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint4* ws;
  uint32_t* out;
  uint64_t* dc;
  CHK(hipMalloc(&ws, (size_t)cus * 4 * 256 * 81 * 16));
  CHK(hipMalloc(&out, (size_t)cus * 4 * 256 * 4));
  CHK(hipMalloc(&dc, (size_t)cus * 16 * 8));
  if (run<2>(cus, ws, out, dc) || run<3>(cus, ws, out, dc) || run<4>(cus, ws, out, dc)) return 1;
  return 0;
}
