// stl_fe25519.h -- GF(2^255-19) arithmetic for the gfx950 verify kernels.
//
// Representation: 9 unsaturated limbs of 29 bits (limb i has weight 2^(29i),
// 261 bits of capacity) held in 32-bit VGPRs.  Chosen by measurement
// (tools/microbench/femul.hip on MI355X): the 9x29 product is 81 pure
// v_mad_u64_u32 column chains with no per-product carry handling and runs
// 1.3x faster than the saturated 8x32 schedule (2.47e11 vs 1.91e11 fe_mul/s
// per GPU), and additions need no carry chain at all.
//
// Limb-bound discipline ("alpha" = max limb / 2^29), checked by the
// STL_FE_BOUNDS build of tests/native:
//   * fe_mul / fe_sq output       alpha <= 1 + 2^-12
//   * fe_carry / fe_sub / fe_neg  alpha <= 1 + 2^-16       (normalised)
//   * fe_add                      alpha = alpha_a + alpha_b (no carry)
//   * fe_mul(a, b) requires  alpha_a * alpha_b <= 7  (each 64-bit column sum
//     of 9 products then stays below 2^64); fe_sq requires alpha^2 <= 7.
//   * fe_sub(a, b) requires alpha_a <= 3.9 and alpha_b <= 3.9.
// Values are only weakly reduced (any representative < 2^262); fe_tobytes /
// fe_iszero / fe_isnegative fully reduce mod p.
//
// Same code compiles for the host (tests/native harness) and the device; it
// is one implementation, not a fallback.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define STL_HD __host__ __device__ __forceinline__

// Limb-bound assertion hooks: empty in the product build; the host test
// harness (tests/native/hostemu.cpp) defines them to count violations.
#ifndef STL_BOUND_MUL
#define STL_BOUND_MUL(a, b)
#define STL_BOUND_SUB(a, b)
#endif

// Scheduling fence after each field multiply: keeps the pre-RA scheduler from
// software-pipelining consecutive products (which multiplies live registers
// and forced spills at 2-4 waves/SIMD).  Device-only hint; no-op on the host.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(STL_NO_FE_FENCE)
#define STL_FE_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define STL_FE_FENCE()
#endif

namespace stl {

constexpr uint32_t M29 = 0x1fffffffu;

struct fe {
  uint32_t v[9];
};

// 4 * Z1, where Z1 = 2^261 - 1216 == 0 (mod p) in 29-bit limbs
// [2^29-1216, 2^29-1, ...]; added before a subtraction so no limb underflows.
#define STL_4Z1_0 0x7fffed00u
#define STL_4Z1_I 0x7ffffffcu

STL_HD void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = 0;
}

STL_HD void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}

// One parallel carry pass: limb_i = (limb_i & M) + (limb_{i-1} >> 29);
// bits >= 2^261 of limb 8 fold into limb 0 with weight 2^261 == 1216 (mod p).
STL_HD void fe_carry(fe& h) {
  uint32_t c[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) c[i] = h.v[i] >> 29;
#pragma unroll
  for (int i = 8; i > 0; --i) h.v[i] = (h.v[i] & M29) + c[i - 1];
  h.v[0] = (h.v[0] & M29) + c[8] * 1216u;
}

STL_HD void fe_add(fe& h, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = a.v[i] + b.v[i];
}

STL_HD void fe_sub(fe& h, const fe& a, const fe& b) {
  STL_BOUND_SUB(a, b);
  h.v[0] = a.v[0] + STL_4Z1_0 - b.v[0];
#pragma unroll
  for (int i = 1; i < 9; ++i) h.v[i] = a.v[i] + STL_4Z1_I - b.v[i];
  fe_carry(h);
}

STL_HD void fe_neg(fe& h, const fe& a) {
  h.v[0] = STL_4Z1_0 - a.v[0];
#pragma unroll
  for (int i = 1; i < 9; ++i) h.v[i] = STL_4Z1_I - a.v[i];
  fe_carry(h);
}

// h = c ? b : a  (lane-wise select, no branch)
STL_HD void fe_cmov(fe& h, const fe& a, const fe& b, bool c) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = c ? b.v[i] : a.v[i];
}

// Product-scanning reduction shared by fe_mul / fe_sq.  COL(k, init) yields
// init + the 64-bit sum of the partial products of column k (k = 0..16, each
// sum < 63 * 2^58).  Fold by register halves: the high columns 9..16 are kept as raw 64-bit sums
// and folded into the low columns by their 32-bit register halves (no 29-bit
// normalisation chain for them): the low half of column k+9 enters column k
// with weight 2^261 == 1216, the high half enters column k+1 with weight
// 2^(261+32-29) == 1216*8 = 9728.  Each low column then starts its mad chain
// from (carry + the two fold terms), so a column costs its products plus one
// and + one 64-bit shift.  Bound: column sums <= 63*2^58*(1+2^-12) plus the
// fold terms < 2^46 stay below 2^64.  Measured on MI355X against the earlier
// schedule that normalised columns 9..16 to 29-bit digits first (one and, one
// 64-bit shift and one 64-bit add per column): 98 vs 91 mads but 22 vs 57 other
// instructions per multiply; verify kernel 14.09 -> 13.31 ms per 1M.
#define STL_FE_REDUCE_COLUMNS(h, COL)                                    \
  do {                                                                  \
    uint64_t hc_[8];                                                    \
    _Pragma("unroll") for (int k = 9; k < 17; ++k) hc_[k - 9] = COL(k, 0ull); \
    uint64_t carry_ = 0;                                                \
    _Pragma("unroll") for (int k = 0; k < 9; ++k) {                     \
      uint64_t init_ = carry_;                                          \
      if (k < 8) init_ += (uint64_t)(uint32_t)hc_[k < 8 ? k : 0] * 1216u; \
      if (k > 0) init_ += (uint64_t)(uint32_t)(hc_[k > 0 ? k - 1 : 0] >> 32) * 9728u; \
      const uint64_t t_ = COL(k, init_);                                \
      (h).v[k] = (uint32_t)t_ & M29;                                    \
      carry_ = t_ >> 29;                                                \
    }                                                                   \
    /* carry_ < 2^35 has weight 2^261 == 1216 */                        \
    const uint64_t u_ = (uint64_t)(h).v[0] + carry_ * 1216u;            \
    (h).v[0] = (uint32_t)u_ & M29;                                      \
    (h).v[1] += (uint32_t)(u_ >> 29);                                   \
  } while (0)


STL_HD uint64_t fe_mul_col(const fe& a, const fe& b, int k, uint64_t acc) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = k - i;
    if (j < 0 || j > 8) continue;
    acc += (uint64_t)a.v[i] * b.v[j];
  }
  return acc;
}

// d = 2a (precomputed); column k of a^2 = sum_{i<j} d_i a_j + [k even] a_{k/2}^2
STL_HD uint64_t fe_sq_col(const fe& a, const uint32_t d[9], int k, uint64_t acc) {
  if ((k & 1) == 0) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = k - i;
    if (j <= i || j > 8) continue;
    acc += (uint64_t)d[i] * a.v[j];
  }
  return acc;
}

STL_HD void fe_mul(fe& h, const fe& a, const fe& b) {
  STL_BOUND_MUL(a, b);
  const fe a_ = a, b_ = b;  // h may alias a or b
#define STL_MUL_COL(k, init) fe_mul_col(a_, b_, (k), (init))
  STL_FE_REDUCE_COLUMNS(h, STL_MUL_COL);
#undef STL_MUL_COL
  STL_FE_FENCE();
}

STL_HD void fe_sq(fe& h, const fe& a) {
  STL_BOUND_MUL(a, a);
  const fe a_ = a;
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = a_.v[i] << 1;  // alpha <= 2.64 => fits 32 bits
#define STL_SQ_COL(k, init) fe_sq_col(a_, d, (k), (init))
  STL_FE_REDUCE_COLUMNS(h, STL_SQ_COL);
#undef STL_SQ_COL
  STL_FE_FENCE();
}

STL_HD void fe_sqn(fe& h, const fe& a, int n) {
  fe_sq(h, a);
#pragma unroll 1
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

// 255-bit little-endian integer in 8 LE 32-bit words -> limbs (bit 255 ignored,
// no reduction: ref10 fe_frombytes semantics).
STL_HD void fe_frombytes(fe& h, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int bit = 29 * i;
    const int wi = bit >> 5, off = bit & 31;
    uint32_t lo = w[wi] >> off;
    uint32_t hi = (off != 0 && wi + 1 < 8) ? (w[wi + 1] << (32 - off)) : 0u;
    h.v[i] = (lo | hi) & M29;
  }
  h.v[8] &= 0x7fffffu;  // bits 232..254
}

// Full reduction to the canonical representative in [0, p), packed into 8 words.
STL_HD void fe_tobytes(uint32_t w[8], const fe& f) {
  fe h = f;
  // exact sequential normalisation (value < 2^262 on entry)
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      uint32_t t = h.v[i] + carry;
      h.v[i] = t & M29;
      carry = t >> 29;
    }
    h.v[0] += carry * 1216u;
  }
  // fold bits >= 255 (limb 8 bits 23..28) with 2^255 == 19, twice
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t top = h.v[8] >> 23;
    h.v[8] &= 0x7fffffu;
    h.v[0] += top * 19u;
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      uint32_t t = h.v[i] + carry;
      h.v[i] = t & M29;
      carry = t >> 29;
    }
  }
  // now h < 2^255; subtract p if h >= p  (h >= p  <=>  h + 19 >= 2^255)
  uint32_t t[9];
  uint32_t carry = 19;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint32_t s = h.v[i] + carry;
    t[i] = s & M29;
    carry = s >> 29;
  }
  const bool ge_p = (t[8] >> 23) != 0;
  t[8] &= 0x7fffffu;
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = ge_p ? t[i] : h.v[i];
  // pack 255 bits
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int bit = 32 * k;
    const int li = bit / 29, off = bit % 29;
    uint32_t v = h.v[li] >> off;
    if (li + 1 < 9) v |= h.v[li + 1] << (29 - off);
    if (off > 26 && li + 2 < 9) v |= h.v[li + 2] << (58 - off);
    w[k] = v;
  }
}

STL_HD bool fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_tobytes(w, f);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d |= w[i];
  return d == 0;
}

STL_HD uint32_t fe_isnegative(const fe& f) {
  uint32_t w[8];
  fe_tobytes(w, f);
  return w[0] & 1u;
}

// z^(p-2) and z^((p-5)/8): the ref10 addition chains (254 / 250 squarings).
STL_HD void fe_invert(fe& out, const fe& z) {
  fe t0, t1, t2, t3;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(t1, z, t1);
  fe_mul(t0, t0, t1);
  fe_sq(t2, t0);
  fe_mul(t1, t1, t2);
  fe_sqn(t2, t1, 5);
  fe_mul(t1, t2, t1);
  fe_sqn(t2, t1, 10);
  fe_mul(t2, t2, t1);
  fe_sqn(t3, t2, 20);
  fe_mul(t2, t3, t2);
  fe_sqn(t2, t2, 10);
  fe_mul(t1, t2, t1);
  fe_sqn(t2, t1, 50);
  fe_mul(t2, t2, t1);
  fe_sqn(t3, t2, 100);
  fe_mul(t2, t3, t2);
  fe_sqn(t2, t2, 50);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 5);
  fe_mul(out, t1, t0);
}

STL_HD void fe_pow22523(fe& out, const fe& z) {
  fe t0, t1, t2;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(t1, z, t1);
  fe_mul(t0, t0, t1);
  fe_sq(t0, t0);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 100);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 50);
  fe_mul(t0, t1, t0);
  fe_sqn(t0, t0, 2);
  fe_mul(out, t0, z);
}

// Curve constants in 29-bit limbs.
STL_HD void fe_const_d(fe& h) {
  const uint32_t c[9] = {0x135978a3u, 0x0f5a6e50u, 0x10762addu, 0x00149a82u, 0x1e898007u,
                         0x003cbbbcu, 0x19ce331du, 0x1dc56dffu, 0x0052036cu};
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = c[i];
}

STL_HD void fe_const_2d(fe& h) {
  const uint32_t c[9] = {0x06b2f159u, 0x1eb4dca1u, 0x00ec55bau, 0x00293505u, 0x1d13000eu,
                         0x00797779u, 0x139c663au, 0x1b8adbffu, 0x002406d9u};
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = c[i];
}

STL_HD void fe_const_sqrtm1(fe& h) {
  const uint32_t c[9] = {0x0a0ea0b0u, 0x0770d93au, 0x0bf91e31u, 0x06300d5au, 0x1d7a72f4u,
                         0x004c9efdu, 0x1c2cad34u, 0x1009f83bu, 0x002b8324u};
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = c[i];
}

}  // namespace stl
