// Where the compiler puts s_nop hazard slots between v_mad_u64_u32 chains on
// gfx950 (distance-4, -3 and -2 chains of independent mads; a multiplicand
// produced by a mad).  hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S
// mad_hazard.hip, then grep v_mad_u64_u32 / s_nop: the slots appear after every
// second mad even when no operand of the next mad was written by the two before.
#include <hip/hip_runtime.h>
#include <stdint.h>
#define F(a) asm volatile("" : "+v"(a))
__global__ void k(uint64_t* o, const uint32_t* x) {
  uint32_t a = x[threadIdx.x], b = x[threadIdx.x + 64], c = x[threadIdx.x + 128], d = x[threadIdx.x+192];
  uint64_t p = 0, q = 0, r = 0, s = 0;
  // distance 4 chain
  for (int i = 0; i < 4; ++i) {
    p += (uint64_t)a * b; F(p);
    q += (uint64_t)b * c; F(q);
    r += (uint64_t)c * d; F(r);
    s += (uint64_t)d * a; F(s);
  }
  // distance 3
  for (int i = 0; i < 4; ++i) {
    p += (uint64_t)a * b; F(p);
    q += (uint64_t)b * c; F(q);
    r += (uint64_t)c * d; F(r);
  }
  // distance 2
  for (int i = 0; i < 4; ++i) {
    p += (uint64_t)a * b; F(p);
    q += (uint64_t)b * c; F(q);
  }
  // multiplicand produced by a mad64 (low half)
  uint32_t m = (uint32_t)p;
  for (int i = 0; i < 3; ++i) { r += (uint64_t)m * c; F(r); s += (uint64_t)b*d; F(s); q += (uint64_t)a*d; F(q); m = (uint32_t)r; }
  o[threadIdx.x] = p + q + r + s;
}
