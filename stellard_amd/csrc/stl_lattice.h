// stl_lattice.h -- half-size scalars for the exact cofactorless check.
//
// The reference accepts iff encode([S]B - [k]A) == R (libsodium's
// crypto_sign_verify_detached, called at RippleAddress.cpp:196-197).  With Q
// the decoding of a canonical R this is  X := [S]B - [k]A - Q == O.  For any
// d with gcd(d, 8L) = 1 (d odd, 0 < |d| < L), X == O  <=>  [d]X == O, because
// every point of the curve has order dividing 8L.  If moreover c == d*k
// (mod 8L) then [d*k]A == [c]A for every A on the curve (torsion included),
// and [d*S]B == [e]B with e = d*S mod L.  So
//
//     accept  <=>  [e]B - [c]A - [d]Q == O,
//
// exactly, with |c|, |d| ~ 2^128 instead of k ~ 2^253: the doubling chain of
// the Straus loop halves (Antipa et al. 2005; Pornin 2020 for EdDSA).  The
// lattice is taken modulo 8L, not L, so that mixed-order keys keep libsodium's
// cofactorless answer (accept iff 8 | k for A = A0 + T8).
//
// (c, d) comes from the extended Euclidean algorithm on (8L, k), stopped when
// the remainder drops below 2^128 (r_i == t_i * k mod 8L, |t_i| <= 8L/r_{i-1}),
// then made odd in d by combining with the previous row.  The Euclid runs as
// Lehmer rounds (lat_lehmer_round): quotients from the leading 53 bits in
// fp64, each certified to equal the full-precision quotient before it is
// taken, so the row sequence is exactly the one-step-at-a-time Euclid's.  Any
// lane whose (c, d) does not fit the 158-bit budget, or needs a quotient >=
// 2^32, is flagged for the full-length path (verify_full_with_k), which is
// exact for every input.
#pragma once
#include "stl_sc25519.h"

namespace stl {

// |c|, |d| < 2^158: fits 40 signed radix-16 digits with the top one in
// [-8, 7].  The main loop runs a wave-uniform number of positions P (the
// wave's largest need, 33 for almost every lane).
constexpr int kHalfBits = 158;
constexpr int kHalfDigits = 40;

STL_HD uint32_t lat_N(int i) {  // 8L, little-endian words
  const uint32_t w[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u};
  return w[i];
}

template <int NW>
STL_HD double lat_to_double(const uint32_t* w) {
  double d = (double)w[NW - 1];
#pragma unroll
  for (int i = NW - 2; i >= 0; --i) d = d * 4294967296.0 + (double)w[i];
  return d;
}

// x >= 2^128 (8-word value)
STL_HD bool lat_ge128(const uint32_t x[8]) { return (x[4] | x[5] | x[6] | x[7]) != 0; }

// x >= y (8 words)
STL_HD bool lat_ge(const uint32_t x[8], const uint32_t y[8]) {
  bool gt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    gt = gt || (eq && x[i] > y[i]);
    eq = eq && x[i] == y[i];
  }
  return gt || eq;
}

// x -= y (8 words, caller guarantees x >= y)
STL_HD void lat_sub(uint32_t x[8], const uint32_t y[8]) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)x[i] - y[i] - borrow;
    x[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
}

// x += y (8 words, mod 2^256)
STL_HD void lat_add(uint32_t x[8], const uint32_t y[8]) {
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t s = (uint64_t)x[i] + y[i] + carry;
    x[i] = (uint32_t)s;
    carry = s >> 32;
  }
}

// x -= q*y over 8 words; returns true when the exact result is negative (it
// is then left as x - q*y + 2^256, i.e. two's complement).
STL_HD bool lat_mulsub(uint32_t x[8], uint32_t q, const uint32_t y[8]) {
  uint64_t carry = 0;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t p = (uint64_t)q * y[i] + carry;
    carry = p >> 32;
    const uint64_t d = (uint64_t)x[i] - (uint32_t)p - borrow;
    x[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  return (carry + borrow) != 0;
}

// t += q*u over 5 words (magnitudes of the Bezout coefficients, < 2^160);
// returns the carry out of the top word (0 unless the sum overflows).
STL_HD uint32_t lat_muladd5(uint32_t t[5], uint32_t q, const uint32_t u[5]) {
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint64_t s = (uint64_t)q * u[i] + t[i] + carry;
    t[i] = (uint32_t)s;
    carry = s >> 32;
  }
  return (uint32_t)carry;
}

// One Euclidean step on the larger remainder x (x > y >= 2^128):
// x <- x mod y, tx <- tx + q*ty with q = floor(x / y).  ok <- false if q >= 2^32.
STL_HD void lat_step(uint32_t x[8], const uint32_t y[8], uint32_t tx[5], const uint32_t ty[5], bool& ok) {
  const double dx = lat_to_double<8>(x), dy = lat_to_double<8>(y);
  const double ratio = dx / dy;
  double qd = floor(ratio);
  if (qd >= 4294967296.0) {
    ok = false;
    qd = 0.0;
  }
  uint32_t q = (uint32_t)qd;
  // |ratio - x/y| < 2^-17 for q < 2^32 (relative error of the two 8-term
  // conversions and the division, each < 2^-50), so floor(ratio) is the
  // true quotient or off by one, and only when ratio is that close to an
  // integer: too large => x - q*y < 0; too small => x - q*y >= y, which is
  // then possible only if ratio - q > 1 - 2^-16.
  const bool neg = lat_mulsub(x, q, y);
  if (neg) {
    lat_add(x, y);
    q -= 1u;
  } else if (ratio - qd > 1.0 - 1.0 / 65536.0) {
    if (lat_ge(x, y)) {
      lat_sub(x, y);
      q += 1u;
    }
  }
  lat_muladd5(tx, q, ty);
}

// 5-word magnitude < 2^kHalfBits
STL_HD bool lat_fits(const uint32_t v[5]) { return (v[4] >> (kHalfBits - 128)) == 0; }

// ---- Lehmer reduction (Knuth 4.5.2 Algorithm L with an exact certificate) ----
// A round reads the leading 53 bits of both rows at one shift, runs Euclid
// on those doubles while each quotient is PROVABLY the full rows' quotient,
// then applies the accumulated 2x2 matrix to the full rows once.  The
// sequence of rows is therefore exactly the one-quotient-per-step Euclid's
// (tests/test_halfscalar.py::test_lattice_equals_exact_euclid), at a
// fraction of the multi-word work.

// wave-uniform loop control: any lane still active (device), this lane (host)
STL_HD bool lat_any(bool b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __any(b);
#else
  return b;
#endif
}

// quotient estimate x / y (corrected exactly by the caller)
STL_HD double lat_div_est(double x, double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  return x * __builtin_amdgcn_rcp(y);
#else
  return x / y;
#endif
}

// Leading parts at a common shift sh: x = floor(r1 / 2^sh) in [2^52, 2^53),
// y = floor(r2 / 2^sh) (exact integers as doubles), and thr = 2^(128 - sh).
// Requires r1 >= 2^128 and r2 < r1 for a meaningful result.
STL_HD void lat_lead(double& x, double& y, double& thr, const uint32_t r1[8], const uint32_t r2[8]) {
  const int t = r1[7] ? 7 : r1[6] ? 6 : r1[5] ? 5 : 4;
  uint32_t a2 = 0, a1 = 0, a0 = 0, b2 = 0, b1 = 0, b0 = 0;
#pragma unroll
  for (int i = 4; i < 8; ++i) {
    if (t == i) {
      a2 = r1[i];
      a1 = r1[i - 1];
      a0 = r1[i - 2];
      b2 = r2[i];
      b1 = r2[i - 1];
      b0 = r2[i - 2];
    }
  }
  const int lz = a2 ? __builtin_clz(a2) : 0;
  uint64_t ta = ((uint64_t)a2 << 32) | a1, tb = ((uint64_t)b2 << 32) | b1;
  if (lz) {
    ta = (ta << lz) | (a0 >> (32 - lz));
    tb = (tb << lz) | (b0 >> (32 - lz));
  }
  x = (double)(ta >> 11);
  y = (double)(tb >> 11);
  thr = ldexp(1.0, 128 - (32 * (t - 2) + 43 - lz));
}

// out = |ua*A - ub*B| computed as neg ? ub*B - ua*A : ua*A - ub*B over nine
// words; bad if that value is negative or >= 2^256 (never, for certified
// quotients; checked all the same, the lane then takes the full-length path).
STL_HD void lat_comb(uint32_t out[8], uint32_t ua, const uint32_t A[8], uint32_t ub, const uint32_t B[8], bool neg,
                     bool& bad) {
  uint64_t ca = 0, cb = 0;
  uint32_t borrow = 0, w[9];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t pa = (uint64_t)ua * A[i] + ca, pb = (uint64_t)ub * B[i] + cb;
    ca = pa >> 32;
    cb = pb >> 32;
    const uint64_t d = (uint64_t)(uint32_t)pa - (uint32_t)pb - borrow;
    w[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  w[8] = (uint32_t)(ca - cb - borrow);
  if (neg) {
    uint64_t carry = 1;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const uint64_t s = (uint64_t)(~w[i]) + carry;
      w[i] = (uint32_t)s;
      carry = s >> 32;
    }
  }
  bad = bad || w[8] != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = w[i];
}

// out = ua*A + ub*B over five words; bad on a carry out
STL_HD void lat_madd2(uint32_t out[5], uint32_t ua, const uint32_t A[5], uint32_t ub, const uint32_t B[5], bool& bad) {
  uint64_t ca = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint64_t pa = (uint64_t)ua * A[i] + (ca & 0xffffffffu);
    const uint64_t s = (uint64_t)ub * B[i] + (uint32_t)pa + (ca >> 32);
    out[i] = (uint32_t)s;
    ca = (pa >> 32) + (s >> 32);  // < 2^33
  }
  bad = bad || ca != 0;
}

// One Lehmer round on the rows (larger rl, smaller rs >= 2^128 when act).
// With M = [[m00, m01], [m10, m11]] the product of the certified steps'
// [[q, 1], [1, 0]], (rl, rs) = M (X, Y): X = det*(m11 rl - m01 rs),
// Y = det*(m00 rs - m10 rl), det = (-1)^steps.  Truncating to the leading
// parts leaves |X/2^sh - x| < max(m11, m01) =: M1 and |Y/2^sh - y| < M2 :=
// max(m10, m00), so q = floor(x / y), r = x - q y is the true quotient of
// (X, Y) when  r >= M1 + q M2  and  y - r >= M1 + (q + 1) M2,  and the step
// is taken while the matrix stays below 2^32.  Euclid stops at the first
// remainder below 2^128: the round goes on only while the new remainder is
// certainly >= 2^128, and otherwise ends with the step that may have crossed
// (lattice_half tests the rows exactly), so a lane's last step is a certified
// one too instead of a round of its own through lat_step.
// At most kLehmerSteps certified steps per round: a wave runs each round's
// loop to its slowest lane, and lanes certify 8-30 quotients from 53 bits
// (tools/lattice_sim.cpp, 2,000 waves of random k: 121.6 iterations in 7.03
// rounds per wave uncapped; 95.7 in 7.15 at 16, the rows unchanged -- every
// step is still an exact Euclid step, only some move to the next round).
#ifndef STL_LEHMER_STEPS
#define STL_LEHMER_STEPS 16
#endif
constexpr int kLehmerSteps = STL_LEHMER_STEPS;

STL_HD void lat_lehmer_round(uint32_t rl[8], uint32_t rs[8], uint32_t tl[5], uint32_t ts[5], bool& tl_neg, bool& ok,
                             bool act) {
  double x, y, thr;
  lat_lead(x, y, thr, rl, rs);
  double m00 = 1.0, m01 = 0.0, m10 = 0.0, m11 = 1.0;
  bool go = act, odd = false;
#pragma unroll 1
  for (int it = 0; it < kLehmerSteps; ++it) {
    if (!lat_any(go)) break;
    double q = floor(lat_div_est(x, y));
    double r = fma(-q, y, x);
    if (r < 0.0) {
      q -= 1.0;
      r += y;
    } else if (r >= y) {
      q += 1.0;
      r -= y;
    }
    const double M1 = fmax(m11, m01), M2 = fmax(m10, m00);
    const double n00 = fma(m00, q, m01), n10 = fma(m10, q, m11);
    const double M2n = fmax(n00, n10);
    const bool step = y > 0.0 && r >= 0.0 && r < y && r >= fma(q, M2, M1) && y - r >= fma(q + 1.0, M2, M1) &&
                      M2n < 4294967296.0;
    go = go && step;
    if (go) {
      m01 = m00;
      m00 = n00;
      m11 = m10;
      m10 = n10;
      x = y;
      y = r;
      odd = !odd;
    }
    // the new remainder may be below 2^128: the round ends with this step,
    // and the caller's exact test decides whether another round follows
    go = go && r - M2n >= thr;
  }
  if (!act) return;
  if (m10 != 0.0) {  // at least one certified step: apply M
    const uint32_t u00 = (uint32_t)m00, u01 = (uint32_t)m01, u10 = (uint32_t)m10, u11 = (uint32_t)m11;
    uint32_t X[8], Y[8], TX[5], TY[5];
    bool bad = false;
    lat_comb(X, u11, rl, u01, rs, odd, bad);
    lat_comb(Y, u10, rl, u00, rs, !odd, bad);
    lat_madd2(TX, u11, tl, u01, ts, bad);
    lat_madd2(TY, u10, tl, u00, ts, bad);
    bad = bad || lat_ge(Y, X);
    ok = ok && !bad;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      rl[i] = X[i];
      rs[i] = Y[i];
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      tl[i] = TX[i];
      ts[i] = TY[i];
    }
    tl_neg = tl_neg != odd;
  } else {  // no certified quotient (large or near-boundary): one exact step
    lat_step(rl, rs, tl, ts, ok);  // rl <- rl mod rs, tl <- tl + q ts
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t v = rl[i];
      rl[i] = rs[i];
      rs[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const uint32_t v = tl[i];
      tl[i] = ts[i];
      ts[i] = v;
    }
    tl_neg = !tl_neg;
  }
}

// (c, d) with c == d*k (mod 8L), d odd, |c|, |d| < 2^158, as magnitudes and
// signs.  Returns false when the lane must take the full-length path.
STL_HD bool lattice_half(uint32_t c[5], bool& c_neg, uint32_t d[5], bool& d_neg, const uint32_t k[8]) {
  // Rows (r, t) with r == t*k (mod 8L): larger (rl, tl), smaller (rs, ts),
  // t as magnitudes; the signs alternate, tl is negative iff tl_neg.
  uint32_t rl[8], rs[8], tl[5], ts[5];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    rl[i] = lat_N(i);
    rs[i] = k[i];
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    tl[i] = 0;
    ts[i] = i == 0 ? 1u : 0u;
  }
  bool ok = true, tl_neg = true;
  // Lehmer rounds (lat_lehmer_round): ~7 per lane for a random k, each
  // certifying ~15 quotients from the leading 53 bits; a round that
  // certifies none takes one exact step, so every round makes progress and
  // 128 rounds exceed the longest Euclid sequence (~180 steps).
#pragma unroll 1
  for (int round = 0; round < 128; ++round) {
    const bool act = ok && lat_ge128(rs);
    if (!lat_any(act)) break;
    lat_lehmer_round(rl, rs, tl, ts, tl_neg, ok, act);
  }
  ok = ok && !lat_ge128(rs);
  const bool ts_neg = !tl_neg;
  if (ts[0] & 1u) {
    // (c, d) = (rs, +-ts): |rs| < 2^128, |ts| <= 8L / rl < 2^128
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      c[i] = rs[i];
      d[i] = ts[i];
    }
    c_neg = false;
    d_neg = ts_neg;
  } else {
    // ts even => tl odd.  w = row_l - j * row_s keeps d odd; the j balancing
    // |rl - j rs| against |tl| + j |ts| gives max-norm ~ 8L / (rs + |ts|).
    const double num = lat_to_double<8>(rl) - lat_to_double<5>(tl);
    const double den = lat_to_double<8>(rs) + lat_to_double<5>(ts);
    double jd = floor(num / den + 0.5);
    if (!(jd >= 0.0)) jd = 0.0;
    if (jd >= 4294967296.0) {
      ok = false;
      jd = 0.0;
    }
    const uint32_t j = (uint32_t)jd;
    uint32_t cw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) cw[i] = rl[i];
    const bool neg = lat_mulsub(cw, j, rs);  // rl - j*rs, two's complement
    if (neg) {  // magnitude = -cw
      uint64_t carry = 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint64_t s = (uint64_t)(~cw[i]) + carry;
        cw[i] = (uint32_t)s;
        carry = s >> 32;
      }
    }
    ok = ok && (cw[5] | cw[6] | cw[7]) == 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      c[i] = cw[i];
      d[i] = tl[i];
    }
    ok = ok && lat_muladd5(d, j, ts) == 0;  // |tl| + j |ts|
    c_neg = neg;
    d_neg = tl_neg;
  }
  return ok && lat_fits(c) && lat_fits(d);
}

// out = d * S mod L for d = (-1)^d_neg * |d|, |d| < 2^160, S < 2^256.
STL_HD void sc_mul_signed(uint32_t out[8], const uint32_t d[5], bool d_neg, const uint32_t S[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t t = (uint64_t)d[i] * S[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  sc_reduce64(out, x);
  // negate mod L when d < 0 (0 stays 0)
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) nz |= out[i];
  if (d_neg && nz != 0) {
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t t = (uint64_t)sc_L(i) - out[i] - borrow;
      out[i] = (uint32_t)t;
      borrow = (uint32_t)(t >> 63);
    }
  }
}

// Signed radix-16 recoding of a magnitude v < 2^158 into 40 digits in
// [-8, 7], packed 4-bit two's complement (digit 8m+j in bits 4j..4j+3 of word
// m).  Returns the number of positions the value needs: 1 + the index of its
// highest nonzero digit (at least 1).
STL_HD int sc_recode16_half(uint32_t packed[5], const uint32_t v[5]) {
  int carry = 0, need = 1;
#pragma unroll
  for (int m = 0; m < 5; ++m) {
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int e = (int)((v[m] >> (4 * j)) & 15u) + carry;
      carry = (e + 8) >> 4;
      e -= carry << 4;
      word |= ((uint32_t)e & 15u) << (4 * j);
      need = e != 0 ? 8 * m + j + 1 : need;
    }
    packed[m] = word;
  }
  return need;
}

}  // namespace stl
