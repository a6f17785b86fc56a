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
// then made odd in d by combining with the previous row.  Quotients are taken
// from fp64 approximations and corrected exactly.  Any lane whose (c, d) does
// fit the 158-bit budget, or needs a quotient >= 2^32, is flagged for the
// full-length path (verify_full_with_k), which is exact for every input.
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

// (c, d) with c == d*k (mod 8L), d odd, |c|, |d| < 2^158, as magnitudes and
// signs.  Returns false when the lane must take the full-length path.
STL_HD bool lattice_half(uint32_t c[5], bool& c_neg, uint32_t d[5], bool& d_neg, const uint32_t k[8]) {
  // slot a: (ra, -ta) -- t in slot a is always <= 0; slot b: (rb, +tb) >= 0
  uint32_t ra[8], rb[8], ta[5], tb[5];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ra[i] = lat_N(i);
    rb[i] = k[i];
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    ta[i] = 0;
    tb[i] = i == 0 ? 1u : 0u;
  }
  bool ok = true;
  bool small_in_a = false;  // which slot holds the remainder < 2^128 at exit
  // At most ~1.44 * 125 steps reduce a 253-bit k to 128 bits (Fibonacci worst
  // case); 192 half-steps bound the loop for every input.
#pragma unroll 1
  for (int it = 0; it < 96; ++it) {
    if (!ok || !lat_ge128(rb)) break;
    lat_step(ra, rb, ta, tb, ok);  // ra < rb now
    if (!ok || !lat_ge128(ra)) {
      small_in_a = true;
      break;
    }
    lat_step(rb, ra, tb, ta, ok);  // rb < ra now
  }
  ok = ok && !(small_in_a ? lat_ge128(ra) : lat_ge128(rb));
  // s = smaller remainder row, l = larger
  uint32_t rs[8], rl[8], ts[5], tl[5];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    rs[i] = small_in_a ? ra[i] : rb[i];
    rl[i] = small_in_a ? rb[i] : ra[i];
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    ts[i] = small_in_a ? ta[i] : tb[i];
    tl[i] = small_in_a ? tb[i] : ta[i];
  }
  const bool ts_neg = small_in_a, tl_neg = !small_in_a;
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
