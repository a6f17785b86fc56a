// stl_sc25519.h -- scalars mod L = 2^252 + 27742317777372353535851937790883648493.
//
// sc_reduce64: the 512-bit k-hash mod L (libsodium sc25519_reduce, called in
// crypto_sign_verify_detached after hashing R||A||M).  Restated as Barrett
// reduction with 32-bit words (HAC 14.42, b = 2^32, k = 8,
// mu = floor(2^512 / L)), which yields the same canonical residue.
// sc_is_canonical: S < L (sc25519_is_canonical == stellard's
// crypto_sign_check_S_lt_l, RippleAddress.cpp:226-245).
#pragma once
#include "stl_fe25519.h"

namespace stl {

STL_HD uint32_t sc_L(int i) {
  const uint32_t Lw[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
  return Lw[i];
}

STL_HD uint32_t sc_mu(int i) {
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  return mu[i];
}

// true iff s (8 LE words) < L
STL_HD bool sc_lt_L(const uint32_t s[8]) {
  bool lt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    const uint32_t l = sc_L(i);
    lt = lt || (eq && s[i] < l);
    eq = eq && s[i] == l;
  }
  return lt;
}

// r (9 words) -= L if r >= L
STL_HD void sc_csub_L(uint32_t r[9]) {
  uint32_t t[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)r[i] - (i < 8 ? sc_L(i) : 0u) - borrow;
    t[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  const bool ge = borrow == 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) r[i] = ge ? t[i] : r[i];
}

// out = x mod L, x = 512-bit integer as 16 LE words
STL_HD void sc_reduce64(uint32_t out[8], const uint32_t x[16]) {
  // q1 = floor(x / b^7): words 7..15 (9 words)
  // q3 = floor(q1 * mu / b^9)
  uint32_t prod[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) prod[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const uint64_t t = (uint64_t)x[7 + i] * sc_mu(j) + prod[i + j] + carry;
      prod[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    prod[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * L) mod b^9, q3 = prod[9..17]
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i + j >= 9) break;
      const uint64_t t = (uint64_t)prod[9 + i] * sc_L(j) + r2[i + j] + carry;
      r2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    if (i + 8 < 9) r2[i + 8] += (uint32_t)carry;
  }
  // r = (x mod b^9) - r2  (mod b^9); then at most two subtractions of L
  uint32_t r[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  sc_csub_L(r);
  sc_csub_L(r);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = r[i];
}

// Signed radix-16 recoding of a scalar < 2^253 into 64 digits in [-8, 8],
// packed as 4-bit two's complement, 8 digits per word (digit 8m+j in bits
// 4j..4j+3 of word m).  Digits 0..62 lie in [-8, 7]; digit 63 in [0, 2].
STL_HD void sc_recode16(uint32_t packed[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int e = (int)((s[m] >> (4 * j)) & 15u) + carry;
      carry = (e + 8) >> 4;
      e -= carry << 4;
      word |= ((uint32_t)e & 15u) << (4 * j);
    }
    packed[m] = word;
  }
}

// Signed radix-256 recoding of a scalar < 2^253 into 32 digits in [-128, 127]
// (digit 31 in [0, 32]), packed as int8, 4 digits per word (digit 4m+j in
// byte j of word m).  Drives the [S]B part with the 128-entry base table.
STL_HD void sc_recode256(uint32_t packed[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int e = (int)((s[m] >> (8 * j)) & 255u) + carry;
      carry = (e + 128) >> 8;
      e -= carry << 8;
      word |= ((uint32_t)e & 255u) << (8 * j);
    }
    packed[m] = word;
  }
}

// Signed radix-2^16 recoding of a scalar < 2^253 into 16 digits in
// [-32768, 32767] (digit 15 in [0, 2^13]), packed as int16, 2 digits per word
// (digit 2m+j in bits 16j..16j+15 of word m).  Drives the [e]B part of the
// half-size check with the two 32769-entry wide base tables.
STL_HD void sc_recode65536(uint32_t packed[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int e = (int)((s[m] >> (16 * j)) & 0xffffu) + carry;
      carry = (e + 32768) >> 16;
      e -= carry << 16;
      word |= ((uint32_t)e & 0xffffu) << (16 * j);
    }
    packed[m] = word;
  }
}

// out = (a*b + c) mod L   (signing: S = r + k*a)
STL_HD void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t p[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) p[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t t = (uint64_t)a[i] * b[j] + p[i + j] + carry;
      p[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    p[i + 8] = (uint32_t)carry;
  }
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint64_t t = (uint64_t)p[i] + (i < 8 ? c[i] : 0u) + carry;
    p[i] = (uint32_t)t;
    carry = t >> 32;
  }
  sc_reduce64(out, p);
}

}  // namespace stl
