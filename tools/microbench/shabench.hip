// SHA-512 compression throughput on gfx950 without memory traffic: each lane
// runs NB compressions on register data.  Reports SIMD-cycles per wave-block
// (time x clock x SIMDs / wave-blocks) for a range of occupancies.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../stellard_amd/csrc/stl_sha512.h"
using namespace stl;

template <int W>
__global__ __launch_bounds__(256, W) void k(uint64_t* out, int nb, uint64_t seed) {
  uint64_t st[8];
  sha512_init(st);
  uint64_t w[16];
  for (int j = 0; j < 16; ++j) w[j] = seed ^ (threadIdx.x * 0x9e3779b97f4a7c15ull) ^ j;
  for (int b = 0; b < nb; ++b) {
    uint64_t x[16];
    for (int j = 0; j < 16; ++j) x[j] = w[j] ^ st[j & 7];
    sha512_compress(st, x);
  }
  uint64_t acc = 0;
  for (int j = 0; j < 8; ++j) acc ^= st[j];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int W>
void run(uint64_t* d, int cus) {
  const int nb = 64;
  const int blocks = cus * W;  // W waves per SIMD: 256-thread blocks = 1 wave per SIMD each
  hipLaunchKernelGGL(k<W>, dim3(blocks), dim3(256), 0, 0, d, nb, 1ull);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<W>, dim3(blocks), dim3(256), 0, 0, d, nb, (uint64_t)r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double wave_blocks = 5.0 * blocks * 4 * nb;
  const double cyc = ms * 1e-3 * 2.4e9 * cus * 4 / wave_blocks;
  printf("W=%d  %.3f ms  %.0f SIMD-cycles per wave-block  %.2f Gblocks/s\n", W, ms / 5, cyc,
         wave_blocks * 64 / (ms * 1e-3) / 1e9);
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  uint64_t* d; hipMalloc(&d, 1 << 24);
  run<1>(d, p.multiProcessorCount);
  run<2>(d, p.multiProcessorCount);
  run<4>(d, p.multiProcessorCount);
  run<6>(d, p.multiProcessorCount);
  run<8>(d, p.multiProcessorCount);
  return 0;
}
