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
#define STL_BOUND_SUBK(a, b, K)
#endif

// Scheduling fence after each field multiply: keeps the pre-RA scheduler from
// software-pipelining consecutive products (which multiplies live registers
// and forced spills at 2-4 waves/SIMD).  Device-only hint; no-op on the host.
#if defined(__HIP_DEVICE_COMPILE__)
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

// Lazy (carry-free) forms.  fe_sub_nc<K>: h = a + K*Z1 - b, no carry pass;
// requires every limb of b <= the matching limb of K*Z1 (alpha_b < K) and
// alpha_a + K < 8 (no 32-bit overflow); output alpha <= alpha_a + K.  Used
// where the consumer is a multiply whose alpha product stays <= 7
// (bounds annotated at each call site in stl_ge25519.h).
template <int K>
STL_HD void fe_sub_nc(fe& h, const fe& a, const fe& b) {
  STL_BOUND_SUBK(a, b, K);
  h.v[0] = a.v[0] + (uint32_t)K * 0x1ffffb40u - b.v[0];
#pragma unroll
  for (int i = 1; i < 9; ++i) h.v[i] = a.v[i] + (uint32_t)K * M29 - b.v[i];
}

// h = K*Z1 - a, no carry pass (alpha_a < K); output alpha <= K.
template <int K>
STL_HD void fe_neg_nc(fe& h, const fe& a) {
  fe z;
  fe_0(z);
  fe_sub_nc<K>(h, z, a);
}

// h = c ? b : a  (lane-wise select, no branch)
STL_HD void fe_cmov(fe& h, const fe& a, const fe& b, bool c) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = c ? b.v[i] : a.v[i];
}

// ---- multiplication -------------------------------------------------------
// Products are scheduled by hand for gfx950: a fixed order that overlaps
// independent v_mad_u64_u32 chains:
//
//   * every column is one mad chain that STARTS from its carry-in / fold
//     terms (no 64-bit re-association add at the end of the chain, which the
//     compiler otherwise inserts to shorten the critical path);
//   * the high column k+11 (a chain from zero) runs alongside low column k;
//   * NOPS independent products (two squarings of a doubling, two products
//     of an addition) are interleaved mad by mad, so each wave always has 2-4
//     independent chains in flight -- a wave issues a mad64 only every ~9
//     cycles (tools/microbench/isarate.hip) and a SIMD holds two waves.
//
// The order is pinned by an empty asm on each accumulator after each mad
// (madf / STL_ACC_FENCE); the compiler still allocates registers and schedules every
// other instruction.  On the host the fence is a no-op and the result is the
// same integer arithmetic.
//
// Reduction ("fold by halves"): the high columns 9..16 are kept as raw 64-bit
// sums and folded into the low columns by their 32-bit register halves: the
// low half of column k+9 enters column k with weight 2^261 == 1216, the high
// half enters column k+1 with weight 2^(261+32-29) == 9728.  Bound: column
// sums <= 63*2^58*(1+2^-12) plus the fold terms < 2^46 stay below 2^64.
// Measured on MI355X (tools/microbench/isarate.hip, SIMD cycles per product
// at 2 waves/SIMD): the compiler-scheduled fold 580 (mul) / 457 (sq); this
// schedule 569 / 442 alone and 545 / 408 per product when two are paired.
#if defined(__HIP_DEVICE_COMPILE__)
#define STL_ACC_FENCE(acc) asm volatile("" : "+v"(acc))
#else
#define STL_ACC_FENCE(acc)
#endif

// One multiply-accumulate term of a column chain.
STL_HD void madf(uint64_t& acc, uint32_t x, uint32_t y) {
  acc += (uint64_t)x * y;
  STL_ACC_FENCE(acc);
}

// Operands of one product: a*b (SQ = false) or a^2 with d = 2a (SQ = true).
template <bool SQ>
struct ProdSrc {
  uint32_t a[9], b[9];  // b = a (SQ: b holds d = 2a)
};

// Number of terms of column k, and term t = (x, y) of column k.
template <bool SQ>
STL_HD constexpr int col_terms(int k) {
  const int lo = k > 8 ? k - 8 : 0;
  if (!SQ) return (k < 8 ? k : 8) - lo + 1;
  const int pairs = k >= 1 ? (k - 1) / 2 - lo + 1 : 0;  // i < j, i + j = k
  return (pairs > 0 ? pairs : 0) + ((k & 1) == 0 ? 1 : 0);
}

template <bool SQ>
STL_HD void col_term(const ProdSrc<SQ>& s, int k, int t, uint32_t& x, uint32_t& y) {
  const int lo = k > 8 ? k - 8 : 0;
  if (!SQ) {
    const int i = lo + t;
    x = s.a[i];
    y = s.b[k - i];
  } else if ((k & 1) == 0 && t == 0) {
    x = s.a[k >> 1];
    y = s.a[k >> 1];
  } else {
    const int i = lo + t - ((k & 1) == 0 ? 1 : 0);
    x = s.b[i];  // 2 a_i
    y = s.a[k - i];
  }
}

// Run up to eight column chains (chain c: product c % NOPS, column kcol[c];
// kcol < 0 = none) round-robin, term by term, accumulating into acc[c].
template <bool SQ, int NOPS>
STL_HD void run_cols(const ProdSrc<SQ>* src, uint64_t* acc, const int* kcol, int nch) {
  int len[8], mx = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    len[c] = (c < nch && kcol[c] >= 0) ? col_terms<SQ>(kcol[c]) : 0;
    mx = len[c] > mx ? len[c] : mx;
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    if (t >= mx) break;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (c >= nch || t >= len[c]) continue;
      uint32_t x, y;
      col_term<SQ>(src[c % NOPS], kcol[c], t, x, y);
      madf(acc[c], x, y);
    }
  }
}

// h[j] = product j (mod p), j < NOPS <= 4, alpha <= 1 + 2^-12 (as fe_mul /
// fe_sq; same input bounds).  Phase P0 runs columns 9 and 10 of every
// product; phase Pk (k = 0..8) runs low column k alongside high column k+11
// (k <= 5).  Low column k starts from carry, then lo(col k+9)*1216 and
// hi(col k+8)*9728 (2^261 == 1216, 2^(261+3) == 9728 mod p).
template <bool SQ, int NOPS>
STL_HD void fe_prod_n(fe* h, const ProdSrc<SQ>* src) {
  uint64_t hc[NOPS][8];  // high columns 9..16 (about four live at a time)
  {
    uint64_t acc[8];
    int kc[8];
#pragma unroll
    for (int c = 0; c < 2 * NOPS; ++c) {
      acc[c] = 0;
      kc[c] = 9 + c / NOPS;
    }
    run_cols<SQ, NOPS>(src, acc, kc, 2 * NOPS);
#pragma unroll
    for (int c = 0; c < 2 * NOPS; ++c) hc[c % NOPS][c / NOPS] = acc[c];
  }
  uint64_t carry[NOPS];
#pragma unroll
  for (int j = 0; j < NOPS; ++j) carry[j] = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    uint64_t acc[8];
    int kc[8];
    const bool hi = k + 11 <= 16;
#pragma unroll
    for (int j = 0; j < NOPS; ++j) {
      acc[j] = carry[j];
      kc[j] = k;
      acc[NOPS + j] = 0;
      kc[NOPS + j] = hi ? k + 11 : -1;
    }
#pragma unroll
    for (int j = 0; j < NOPS; ++j)
      if (k < 8) madf(acc[j], (uint32_t)hc[j][k], 1216u);
#pragma unroll
    for (int j = 0; j < NOPS; ++j)
      if (k > 0) madf(acc[j], (uint32_t)(hc[j][k - 1] >> 32), 9728u);
    run_cols<SQ, NOPS>(src, acc, kc, hi ? 2 * NOPS : NOPS);
#pragma unroll
    for (int j = 0; j < NOPS; ++j) {
      h[j].v[k] = (uint32_t)acc[j] & M29;
      carry[j] = acc[j] >> 29;
      if (hi) hc[j][k + 2] = acc[NOPS + j];
    }
  }
#pragma unroll
  for (int j = 0; j < NOPS; ++j) {
    const uint64_t u = (uint64_t)h[j].v[0] + carry[j] * 1216u;
    h[j].v[0] = (uint32_t)u & M29;
    h[j].v[1] += (uint32_t)(u >> 29);
  }
}

// Entry points: one product (fe_mul, fe_sq) or two interleaved (fe_mul2, fe_sq2).
STL_HD void fe_mul2(fe& h0, const fe& a0, const fe& b0, fe& h1, const fe& a1, const fe& b1) {
  STL_BOUND_MUL(a0, b0);
  STL_BOUND_MUL(a1, b1);
  ProdSrc<false> s[2];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    s[0].a[i] = a0.v[i];
    s[0].b[i] = b0.v[i];
    s[1].a[i] = a1.v[i];
    s[1].b[i] = b1.v[i];
  }
  fe h[2];
  fe_prod_n<false, 2>(h, s);
  h0 = h[0];
  h1 = h[1];
  STL_FE_FENCE();
}

STL_HD void fe_sq2(fe& h0, const fe& a0, fe& h1, const fe& a1) {
  STL_BOUND_MUL(a0, a0);
  STL_BOUND_MUL(a1, a1);
  ProdSrc<true> s[2];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    s[0].a[i] = a0.v[i];
    s[0].b[i] = a0.v[i] << 1;
    s[1].a[i] = a1.v[i];
    s[1].b[i] = a1.v[i] << 1;
  }
  fe h[2];
  fe_prod_n<true, 2>(h, s);
  h0 = h[0];
  h1 = h[1];
  STL_FE_FENCE();
}

// N independent products interleaved (N <= 4): with three or four chains in
// flight a dependent mad is always >= 3 instructions after its predecessor,
// so no hazard s_nop is needed and each wave keeps 3-4 mads in flight.
template <int N>
STL_HD void fe_mul_n(fe* h, const fe* const* a, const fe* const* b) {
  ProdSrc<false> s[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    STL_BOUND_MUL(*a[j], *b[j]);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      s[j].a[i] = a[j]->v[i];
      s[j].b[i] = b[j]->v[i];
    }
  }
  fe_prod_n<false, N>(h, s);
  STL_FE_FENCE();
}

template <int N>
STL_HD void fe_sq_n(fe* h, const fe* const* a) {
  ProdSrc<true> s[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    STL_BOUND_MUL(*a[j], *a[j]);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      s[j].a[i] = a[j]->v[i];
      s[j].b[i] = a[j]->v[i] << 1;
    }
  }
  fe_prod_n<true, N>(h, s);
  STL_FE_FENCE();
}

STL_HD void fe_mul3(fe& h0, const fe& a0, const fe& b0, fe& h1, const fe& a1, const fe& b1, fe& h2, const fe& a2,
                    const fe& b2) {
  const fe* a[3] = {&a0, &a1, &a2};
  const fe* b[3] = {&b0, &b1, &b2};
  fe h[3];
  fe_mul_n<3>(h, a, b);
  h0 = h[0];
  h1 = h[1];
  h2 = h[2];
}

STL_HD void fe_mul4(fe& h0, const fe& a0, const fe& b0, fe& h1, const fe& a1, const fe& b1, fe& h2, const fe& a2,
                    const fe& b2, fe& h3, const fe& a3, const fe& b3) {
  const fe* a[4] = {&a0, &a1, &a2, &a3};
  const fe* b[4] = {&b0, &b1, &b2, &b3};
  fe h[4];
  fe_mul_n<4>(h, a, b);
  h0 = h[0];
  h1 = h[1];
  h2 = h[2];
  h3 = h[3];
}

STL_HD void fe_sq4(fe& h0, const fe& a0, fe& h1, const fe& a1, fe& h2, const fe& a2, fe& h3, const fe& a3) {
  const fe* a[4] = {&a0, &a1, &a2, &a3};
  fe h[4];
  fe_sq_n<4>(h, a);
  h0 = h[0];
  h1 = h[1];
  h2 = h[2];
  h3 = h[3];
}

STL_HD void fe_mul(fe& h0, const fe& a0, const fe& b0) {
  STL_BOUND_MUL(a0, b0);
  ProdSrc<false> s[1];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    s[0].a[i] = a0.v[i];
    s[0].b[i] = b0.v[i];
  }
  fe h[1];
  fe_prod_n<false, 1>(h, s);
  h0 = h[0];
  STL_FE_FENCE();
}

STL_HD void fe_sq(fe& h0, const fe& a0) {
  STL_BOUND_MUL(a0, a0);
  ProdSrc<true> s[1];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    s[0].a[i] = a0.v[i];
    s[0].b[i] = a0.v[i] << 1;
  }
  fe h[1];
  fe_prod_n<true, 1>(h, s);
  h0 = h[0];
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
