// stl_verify_core.h -- one Ed25519 verification per lane, with the exact
// accept predicate of stellard's RippleAddress::verifySignature
// (src/ripple_data/protocol/RippleAddress.cpp:190-200):
//     crypto_sign_verify_detached(sig, hash, 32, pk) == 0   &&   S < L
// where crypto_sign_verify_detached is libsodium's (not vendored; 1.0.18 is
// the executable oracle here, 1.0.0 is what the reference pins):
//   1.0.18: S < L, R not small order, A canonical, A not small order,
//   both:   A decompresses, k = SHA-512(R||A||M) mod L,
//           accept iff encode([k](-A) + [S]B) == R byte-for-byte (cofactorless)
//   1.0.0:  (sig[63] & 0xE0) == 0 instead of the four 1.0.18 pre-checks.
//
// Scalar multiplication: joint fixed-window (signed radix 16) Straus with
// shared doublings -- uniform control flow across the wave (no per-lane
// sliding-window branches).  Variable points use 9-entry per-lane tables of
// cached multiples (TableView: HBM heads, LDS or HBM tails); [S]B / [e]B use
// constant affine tables of j*B.  The full-length check gives the same group
// element as libsodium's sliding-window ge25519_double_scalarmult_vartime, so
// encode() matches byte-for-byte; the half-size check is exact by the argument
// before verify_phase2_half.
#pragma once
#include "stl_ge25519.h"
#include "stl_sc25519.h"
#include "stl_lattice.h"
#include "stl_sha512.h"
#include "stl_base_table.h"

namespace stl {

enum : uint32_t {
  kPolicySodium1018 = 0u,
  kPolicyStellard100 = 1u,
  // or-ed into a policy: the raw crypto_sign_verify_detached predicate,
  // without stellard's S < L (test-only: RippleAddress.cpp:838-845's raw
  // expectation; STL_DEBUG_RAW_PREDICATE)
  kPolicyRaw = 2u,
};

// stellard's composite accept needs S < L unless the raw predicate is asked for
STL_HD bool composite_s_ok(const uint32_t S[8], uint32_t policy) { return (policy & kPolicyRaw) != 0 || sc_lt_L(S); }

STL_HD uint32_t small_order_word(int e, int i) {
  const uint32_t bl[7][8] = {
      {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
      {0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
      {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du},
      {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u},
      {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu}};
  return bl[e][i];
}

// ge25519_has_small_order: bytes 0..30 and (byte 31 & 0x7f) vs the 7 encodings
STL_HD bool has_small_order(const uint32_t s[8]) {
  bool any = false;
#pragma unroll
  for (int e = 0; e < 7; ++e) {
    bool eq = (s[7] & 0x7fffffffu) == small_order_word(e, 7);
#pragma unroll
    for (int i = 0; i < 7; ++i) eq = eq && s[i] == small_order_word(e, i);
    any = any || eq;
  }
  return any;
}

// ge25519_is_canonical: the 255-bit y is < p
STL_HD bool point_is_canonical(const uint32_t s[8]) {
  bool top = (s[7] & 0x7fffffffu) == 0x7fffffffu;
#pragma unroll
  for (int i = 1; i < 7; ++i) top = top && s[i] == 0xffffffffu;
  return !(top && s[0] >= 0xffffffedu);
}

STL_HD bool all_zero(const uint32_t s[8]) {
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a |= s[i];
  return a == 0;
}

// Pre-checks of crypto_sign_verify_detached for the selected policy.  The
// 1.0.0 policy also rejects the all-zero key, as some 1.0.x releases did (it
// decodes to a point of order 4, for which signatures can be forged).  That
// case is parity-unpinned offline and a reject is the
// safe side: stellard then runs its own serial check.
STL_HD bool verify_prechecks(const uint32_t R[8], const uint32_t S[8], const uint32_t A[8], uint32_t policy) {
  if ((policy & 1u) == kPolicyStellard100) return (S[7] >> 29) == 0 && !all_zero(A);  // sig[63] & 224
  return sc_lt_L(S) && !has_small_order(R) && point_is_canonical(A) && !has_small_order(A);
}

constexpr uint32_t kTableQuadsPerKey = 9 * 9;  // a 9-entry cached table, 9 x uint4 per entry

// Table of cached multiples e*P (9 x uint4 = 144 B per entry).  Quads 0-7 of
// entry e are at main[e * estride + q], quad 8 at tail[e * tstride]:
//   contiguous  one 1,296-B block, entry after entry (estride = tstride = 9):
//               the shared per-key tables of STL_DEDUP_KEYS;
//   split       per-lane tables: the 128-B heads of entries 1-8 in an array
//               of whole lines (estride 8; entry 0's head is a shared
//               identity line) and the 16-B tails apart (in LDS in the main
//               kernel), so a lookup reads one aligned line.
struct TableView {
  uint4* main;
  uint4* tail;
  int estride, tstride;
  // split tables do not store entry 0 (the identity): its head is this one
  // shared line (L2-resident), so the per-lane heads are 8 lines per table
  const uint4* id;
  static STL_HD TableView contiguous(uint4* base) { return TableView{base, base + 8, 9, 9, nullptr}; }
  static STL_HD TableView split(uint4* head, uint4* tails, const uint4* id_head, int tstride = 1) {
    return TableView{head, tails, 8, tstride, id_head};
  }
  STL_HD const uint4* head(int e) const {
#ifdef STL_EXP_TABLE_LINES
    // timing-only (wrong results): a per-lane table of
    // STL_EXP_TABLE_LINES head lines -- entries folded onto them -- bounds
    // what any smaller table layout could gain from its footprint alone
    if (id) return e == 0 ? id : main + ((e - 1) % STL_EXP_TABLE_LINES) * estride;
#endif
    if (id) return e == 0 ? id : main + (e - 1) * estride;
    return main + e * estride;
  }
  STL_HD void store(int e, const ge_cached& c) const {
    uint32_t buf[36];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      buf[i] = c.YpX.v[i];
      buf[9 + i] = c.YmX.v[i];
      buf[18 + i] = c.Z.v[i];
      buf[27 + i] = c.T2d.v[i];
    }
    if (!(id && e == 0)) {
      uint4* h = const_cast<uint4*>(head(e));
#pragma unroll
      for (int q = 0; q < 8; ++q) h[q] = make_uint4(buf[4 * q], buf[4 * q + 1], buf[4 * q + 2], buf[4 * q + 3]);
    }
    tail[e * tstride] = make_uint4(buf[32], buf[33], buf[34], buf[35]);
  }
  STL_HD void load(int e, ge_cached& c) const {
    uint32_t buf[36];
    const uint4* h = head(e);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const uint4 v = q < 8 ? h[q] : tail[e * tstride];
      buf[4 * q] = v.x;
      buf[4 * q + 1] = v.y;
      buf[4 * q + 2] = v.z;
      buf[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      c.YpX.v[i] = buf[i];
      c.YmX.v[i] = buf[9 + i];
      c.Z.v[i] = buf[18 + i];
      c.T2d.v[i] = buf[27 + i];
    }
  }
};

// j*B from the 128-entry affine table (row-major, kBaseNielsWords per row):
// absd = |digit| in [0, 128]; digit 0 selects the identity (1, 1, 0).
STL_HD void load_base_niels(ge_niels& n, const uint32_t* tab, int absd) {
  const uint32_t* row = tab + (absd > 0 ? absd - 1 : 0) * 28;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    n.ypx.v[i] = row[i];
    n.ymx.v[i] = row[9 + i];
    n.xy2d.v[i] = row[18 + i];
  }
  ge_niels id;
  fe_1(id.ypx);
  fe_1(id.ymx);
  fe_0(id.xy2d);
  const bool z = absd == 0;
  fe_cmov(n.ypx, n.ypx, id.ypx, z);
  fe_cmov(n.ymx, n.ymx, id.ymx, z);
  fe_cmov(n.xy2d, n.xy2d, id.xy2d, z);
}

// Per-lane table of cached multiples e*P, e = 0..8 (entry 0 = identity), for
// an AFFINE P (Z = 1, T = xy -- every caller's P comes from a decoding or
// affine_to_p3): P's cached form is then its Niels form (Y+X, Y-X, 2dT with
// Z = 1), so 3P..8P are mixed additions (ge_madd, one product fewer than
// ge_add_cached) and 2P skips the square of Z.
STL_HD void build_cached_table(const TableView& tab, const ge_p3& P) {
  ge_cached c1, c;
  ge_cached_0(c);
  tab.store(0, c);
  ge_p3_to_cached(c1, P);
  tab.store(1, c1);
  ge_niels n1;
  n1.ypx = c1.YpX;
  n1.ymx = c1.YmX;
  n1.xy2d = c1.T2d;
  ge_p1p1 t;
  ge_p3 p3;
  ge_affine_dbl(t, P);
  ge_p1p1_to_p3(p3, t);
  ge_p3_to_cached(c, p3);
  tab.store(2, c);
  constexpr int kLast = 8;
#pragma unroll 1
  for (int e = 3; e <= kLast; ++e) {
    ge_madd(t, p3, n1);
    ge_p1p1_to_p3(p3, t);
    ge_p3_to_cached(c, p3);
    tab.store(e, c);
  }
}

// acc + sign(digit) * tab[|digit|], |digit| <= 8
STL_HD void add_table_digit(ge_p1p1& t, const ge_p3& acc, const TableView& tab, int digit) {
  ge_cached c;
  const int a = digit < 0 ? -digit : digit;
  tab.load(a > 8 ? 8 : a, c);
  ge_cached_cneg(c, digit < 0);
  ge_add_cached(t, acc, c);
}

// acc + sign(digit) * btab[|digit|] (affine base table), |digit| <= 128
STL_HD void madd_base_digit(ge_p1p1& t, const ge_p3& acc, const uint32_t* btab, int digit) {
  const int a = digit < 0 ? -digit : digit;
  ge_niels n;
  load_base_niels(n, btab, a > 128 ? 128 : a);
  ge_niels_cneg(n, digit < 0);
  ge_madd(t, acc, n);
}

// acc <- [16] acc2: three p2 doublings and a fourth into p3 (for an add)
STL_HD void dbl4(ge_p3& acc, ge_p2& acc2) {
  ge_p1p1 t;
#pragma unroll 1
  for (int r = 0; r < 3; ++r) {
    ge_p2_dbl<true>(t, acc2);
    ge_p1p1_to_p2(acc2, t);
  }
  ge_p2_dbl(t, acc2);
  ge_p1p1_to_p3(acc, t);
}

// R' = [k](-A) + [S]B  with k, S < 2^253.  negA is the decompressed -A.
// Joint Straus over 64 nibble positions (shared doublings): k in signed
// radix 16 (an A-add at every position, 9-entry per-lane table), S in signed
// radix 256 (a B-add at every even position, 128-entry shared table
// `btab`, LDS on the device).
STL_HD void double_scalarmult(ge_p2& out, const ge_p3& negA, const uint32_t k[8], const uint32_t S[8],
                              const TableView& tab, const uint32_t* btab) {
  build_cached_table(tab, negA);
  // ---- signed digits ----
  uint32_t kd[8], sd[8];
  sc_recode16(kd, k);
  sc_recode256(sd, S);
  // ---- main loop: 64 nibble positions, most significant first ----
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p2 acc2;
  uint32_t wa = 0, wb = 0;
#pragma unroll 1
  for (int i = 63; i >= 0; --i) {
    if ((i & 7) == 7) {  // next 8 radix-16 digits of k
      wa = kd[7];
#pragma unroll
      for (int m = 7; m > 0; --m) kd[m] = kd[m - 1];
    }
    if ((i & 7) == 6) {  // next 4 radix-256 digits of S
      wb = sd[7];
#pragma unroll
      for (int m = 7; m > 0; --m) sd[m] = sd[m - 1];
    }
    if (i != 63) dbl4(acc, acc2);
    // A digit (every position)
    ge_p1p1 t;
    add_table_digit(t, acc, tab, (int32_t)wa >> 28);
    wa <<= 4;
    if (i & 1) {
      ge_p1p1_to_p2(acc2, t);
    } else {
      // B digit (even positions: bits 4i .. 4i+7)
      ge_p1p1_to_p3(acc, t);
      madd_base_digit(t, acc, btab, (int32_t)wb >> 24);
      wb <<= 8;
      ge_p1p1_to_p2(acc2, t);
    }
  }
  out = acc2;
}

// ---- two-phase form used by the gfx950 kernels ----
// Phase 1 (short-lived, few registers): pre-checks, k, decompression of A.
// Phase 2 (the Straus loop, register-heavy): [k](-A) + [S]B, encode, compare.
// Splitting them into two launches keeps each kernel's register allocation to
// what its own phase needs.  PreState is 112 bytes
// (7 x uint4), written and read once per signature.
struct PreState {
  uint32_t k[8];     // H(R||A||M) mod L
  fe negAx, negAy;   // decompressed -A, affine (Z = 1)
  uint32_t ok;       // pre-checks && A decodes && S < L (stellard composite)
  uint32_t pad;
};
static_assert(sizeof(PreState) == 112, "PreState must be 7 x uint4");

STL_HD void verify_phase1(PreState& o, const uint32_t R[8], const uint32_t S[8], const uint32_t A[8],
                          const uint32_t k[8], uint32_t policy) {
  bool ok = verify_prechecks(R, S, A, policy);
  ge_p3 negA;
  ok = ge_frombytes_negate_vartime(negA, A) && ok;
  // stellard composite: && signatureIsCanonical (S < L), RippleAddress.cpp:198-199
  ok = ok && composite_s_ok(S, policy);
#pragma unroll
  for (int i = 0; i < 8; ++i) o.k[i] = k[i];
  o.negAx = negA.X;
  o.negAy = negA.Y;
  o.ok = ok ? 1u : 0u;
  o.pad = 0;
}

STL_HD bool verify_phase2(const PreState& p, const uint32_t R[8], const uint32_t S[8], const TableView& tab,
                          const uint32_t* bniels) {
  ge_p3 negA;
  negA.X = p.negAx;
  negA.Y = p.negAy;
  fe_1(negA.Z);
  fe_mul(negA.T, negA.X, negA.Y);
  // S < 2^253 is guaranteed for accepted lanes under both policies; mask so a
  // rejected lane still runs the same bounded digit range.
  uint32_t Sm[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) Sm[i] = S[i];
  Sm[7] &= 0x1fffffffu;
  ge_p2 Rp;
  double_scalarmult(Rp, negA, p.k, Sm, tab, bniels);
  uint32_t enc[8];
  ge_tobytes(enc, Rp);
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq = eq && enc[i] == R[i];
  return p.ok != 0 && eq;
}

// Full-length check given k = H(R||A||M) mod L (8 words): exact for every
// input; the fallback of the half-size path below.
STL_HD bool verify_full_with_k(const uint32_t R[8], const uint32_t S[8], const uint32_t A[8], const uint32_t k[8],
                               uint32_t policy, const TableView& tab, const uint32_t* bniels) {
  PreState p;
  verify_phase1(p, R, S, A, k, policy);
  return verify_phase2(p, R, S, tab, bniels);
}

// ---- half-size-scalar path (stl_lattice.h): [e]B + [c](-A) + [d](-Q) == O ----
// Phase-1 output, 224 bytes (14 x uint4).  Quads 0-4 (words 0-19) come from
// the scalar half of phase 1, quads 5-13 from the point half:
//   cdig/ddig  signed radix-16 digits 0..39 of |c|, |d| (4-bit packed)
//   tops       bits 0-7: positions needed (max over c, d; 33 for almost
//              every lane), bit 16 ok (pre-checks, decodings, S < L),
//              bit 17 fallback (full-length path); between the two halves
//              bit 17 = "the reduction did not fit", bits 18/19 = sign of
//              c / d
//   edig       signed radix-2^16 digits of e = d*S mod L (16 digits)
//   P1, P2     affine P1 = sign(c) ? A : -A,  P2 = sign(d) ? Q : -Q
struct HalfState {
  uint32_t cdig[5], ddig[5];
  uint32_t tops;
  uint32_t edig[8];
  uint32_t pad;
  fe P1x, P1y, P2x, P2y;
};
static_assert(sizeof(HalfState) == 224, "HalfState must be 14 x uint4");
constexpr int kHalfScalarQuads = 5;  // quads 0-4: digits, tops, pad
constexpr int kHalfTopsWord = 10;
constexpr uint32_t kHalfOk = 1u << 16;
constexpr uint32_t kHalfFallback = 1u << 17;
constexpr uint32_t kHalfCNeg = 1u << 18;
constexpr uint32_t kHalfDNeg = 1u << 19;
// STL_DEDUP_KEYS: the lane's key has a shared per-key table (multiples of -A,
// cached form) at index `pad`; kHalfCNeg is kept so phase 2 can flip the
// digit signs for P1 = +A.
constexpr uint32_t kHalfKeyed = 1u << 20;
// ... and the key also has a wide shared table (j*(-A), j = 0..136, cached
// form): c's digits are taken in pairs as signed radix-256 digits, one A-add
// every second position.
constexpr uint32_t kHalfKeyedWide = 1u << 21;
constexpr int kWideKeyEntries = 137;  // |16*d1 + d0| <= 136 for signed radix-16 digits |d| <= 8

// encode(P) == R is possible for some point P iff R is a canonical encoding:
// y < p, and not "x == 0 with the sign bit set" (x == 0 <=> y == +-1).
STL_HD bool r_is_canonical(const uint32_t R[8]) {
  if (!point_is_canonical(R)) return false;
  const bool sign = (R[7] >> 31) != 0;
  bool one = R[0] == 1u, pm1 = R[0] == 0xffffffecu;
#pragma unroll
  for (int i = 1; i < 7; ++i) {
    one = one && R[i] == 0u;
    pm1 = pm1 && R[i] == 0xffffffffu;
  }
  one = one && (R[7] & 0x7fffffffu) == 0u;
  pm1 = pm1 && (R[7] & 0x7fffffffu) == 0x7fffffffu;
  return !(sign && (one || pm1));
}

// Phase 1, scalar half: k -> (c, d) (lattice_half) -> digits of |c|, |d|
// and e = d*S mod L.  Light on registers and latency-bound (the Euclid
// quotient chain, the SHA-512 rounds of k): its kernel runs at 4 waves/SIMD.
STL_HD void verify_phase1_scalars(HalfState& o, const uint32_t S[8], const uint32_t k[8]) {
  uint32_t c[5], d[5];
  bool c_neg = false, d_neg = false;
  const bool half = lattice_half(c, c_neg, d, d_neg, k);
  uint32_t e[8];
  sc_mul_signed(e, d, d_neg, S);
  const int cneed = sc_recode16_half(o.cdig, c);
  const int dneed = sc_recode16_half(o.ddig, d);
  sc_recode65536(o.edig, e);
  const int need = cneed > dneed ? cneed : dneed;
  o.tops = (uint32_t)need | (half ? 0u : kHalfFallback) | (c_neg ? kHalfCNeg : 0u) | (d_neg ? kHalfDNeg : 0u);
  o.pad = 0;
}

// P1 = sign(c) * A, P2 = sign(d) * Q from the decoded -A, -Q; final flags.
STL_HD void finish_phase1_points(HalfState& o, const fe& nAx, const fe& nAy, const fe& nQx, const fe& nQy, bool ok) {
  const bool c_neg = (o.tops & kHalfCNeg) != 0, d_neg = (o.tops & kHalfDNeg) != 0;
  const bool fits = (o.tops & kHalfFallback) == 0;
  fe nx;
  fe_neg(nx, nAx);
  fe_cmov(o.P1x, nAx, nx, c_neg);
  o.P1y = nAy;
  fe_neg(nx, nQx);
  fe_cmov(o.P2x, nQx, nx, d_neg);
  o.P2y = nQy;
  o.tops = (o.tops & 0xffu) | (ok ? kHalfOk : 0u) | (ok && !fits ? kHalfFallback : 0u);
}

// Phase 1, point half: pre-checks, decompression of A and R (the two
// pow22523 chains, register-heavy), P1 / P2 signed by the scalar half's
// c / d signs, final ok / fallback flags in tops.
STL_HD void verify_phase1_points(HalfState& o, const uint32_t R[8], const uint32_t S[8], const uint32_t A[8],
                                 uint32_t policy) {
  bool ok = verify_prechecks(R, S, A, policy);
  // stellard composite: && signatureIsCanonical (S < L), RippleAddress.cpp:198-199
  ok = ok && composite_s_ok(S, policy) && r_is_canonical(R);  // before the decodings: R, S not live across them
  ge_p3 negA, negQ;
  bool okA, okR;
  // one decoding at a time: 128 VGPRs, 4 waves/SIMD; measured 1-3 % faster
  // than the paired chains at 2 waves
  okA = ge_frombytes_negate_vartime(negA, A);
  okR = ge_frombytes_negate_vartime(negQ, R);
  ok = ok && okA && okR;
  finish_phase1_points(o, negA.X, negA.Y, negQ.X, negQ.Y, ok);
}

// Small batches: verify_phase1_points on a lane pair, one decoding per lane
// (`par` 0 decodes A, 1 decodes R, into -A / -Q); the pair swaps the results
// (verify_prep_pair_kernel); phase1_points_ok gives the pair's flag and
// finish_phase1_points the signed P1 / P2.
STL_HD bool phase1_decode_lane(fe& nx, fe& ny, const uint32_t R[8], const uint32_t A[8], int par) {
  uint32_t P[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) P[i] = par ? R[i] : A[i];
  ge_p3 n;
  const bool ok = ge_frombytes_negate_vartime(n, P);
  nx = n.X;
  ny = n.Y;
  return ok;
}

// The point role's flag (verify_prep_pair_kernel): the pre-checks of the
// policy, stellard's S < L, a canonical R and both decodings.
STL_HD bool phase1_points_ok(const uint32_t R[8], const uint32_t S[8], const uint32_t A[8], uint32_t policy, bool okA,
                             bool okR) {
  return verify_prechecks(R, S, A, policy) && composite_s_ok(S, policy) && r_is_canonical(R) && okA && okR;
}

// Phase 1, point half, with -A decoded once per distinct key of the batch
// (STL_DEDUP_KEYS: many transactions share a signer): decodes only R.  The
// key's decoding is a function of its 32 bytes alone, so the result is the
// same as decoding it in every lane.
STL_HD void verify_phase1_points_keyed(HalfState& o, const uint32_t R[8], const uint32_t S[8], const uint32_t A[8],
                                       uint32_t policy, const fe& negAx, const fe& negAy, bool okA) {
  bool ok = verify_prechecks(R, S, A, policy);
  ok = ok && composite_s_ok(S, policy) && r_is_canonical(R);
  ge_p3 negQ;
  const bool okR = ge_frombytes_negate_vartime(negQ, R);
  ok = ok && okA && okR;
  finish_phase1_points(o, negAx, negAy, negQ.X, negQ.Y, ok);
}

STL_HD void verify_phase1_half(HalfState& o, const uint32_t R[8], const uint32_t S[8], const uint32_t A[8],
                               const uint32_t k[8], uint32_t policy) {
  verify_phase1_scalars(o, S, k);
  verify_phase1_points(o, R, S, A, policy);
}

STL_HD void affine_to_p3(ge_p3& P, const fe& x, const fe& y) {
  P.X = x;
  P.Y = y;
  fe_1(P.Z);
  fe_mul(P.T, x, y);
}

// ---- wide per-key tables in two stages (round 6) ----
// A key's wide table holds j*P, j = 0..136 (P = -A, kWideKeyEntries), in
// cached form.  Stage 1 (one lane per key and i < kWideBaseEntries) builds the
// 24 entries the others are sums of: a*P for a = 0..15 (entry a) and 16b*P
// for b = 1..8 (entry 16b), by double-and-add; stage 2 (one lane per
// remaining entry 16b + a, a = 1..15) adds entry a to entry 16b -- one
// addition instead of the eight doublings and up to eight additions a lane
// spent on its j before (key_table_wide_kernel: 96 us of config 1's 100k-row
// call on the critical path).
constexpr int kWideBaseEntries = 24;
// the entry stage-1 lane i builds
STL_HD int wide_base_index(int i) { return i < 16 ? i : 16 * (i - 15); }

// 1/d (d = -121665/121666), canonical limbs
STL_HD void fe_const_dinv(fe& h) {
  const uint32_t c[9] = {0x0dc9f843u, 0x0f0793b6u, 0x1e550b89u, 0x1bad3084u, 0x1cf660b5u,
                         0x108a66dcu, 0x190cac58u, 0x1a429ab9u, 0x0040907eu};
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = c[i];
}

// j*P for j < 256 by double-and-add over j's bits (P affine), cached form
STL_HD void small_multiple_cached(ge_cached& out, const fe& x, const fe& y, int j) {
  ge_p3 P, acc;
  affine_to_p3(P, x, y);
  ge_cached cP;
  ge_p3_to_cached(cP, P);
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 a2;
#pragma unroll 1
  for (int b = 7; b >= 0; --b) {
    ge_p3_to_p2(a2, acc);
    ge_p2_dbl(t, a2);
    ge_p1p1_to_p3(acc, t);
    if ((j >> b) & 1) {
      ge_add_cached(t, acc, cP);
      ge_p1p1_to_p3(acc, t);
    }
  }
  ge_p3_to_cached(out, acc);
}

// A cached entry (Y+X, Y-X, Z, 2dT) back in extended coordinates, scaled by
// 2: (2X : 2Y : 2Z : 2T) = (YpX - YmX, YpX + YmX, 2Z, T2d / d) -- a valid
// representative of the same point (2X * 2Y == 2Z * 2T), one product.
STL_HD void cached_to_p3x2(ge_p3& r, const ge_cached& c) {
  fe_sub(r.X, c.YpX, c.YmX);
  fe_add(r.Y, c.YpX, c.YmX);
  fe_carry(r.Y);
  fe_add(r.Z, c.Z, c.Z);
  fe_carry(r.Z);
  fe dinv;
  fe_const_dinv(dinv);
  fe_mul(r.T, c.T2d, dinv);
}

// entry 16b + a = entry 16b + entry a (stage 2)
STL_HD void wide_pair_entry(ge_cached& out, const ge_cached& e16b, const ge_cached& ea) {
  ge_p3 P, S;
  cached_to_p3x2(P, e16b);
  ge_p1p1 t;
  ge_add_cached(t, P, ea);
  ge_p1p1_to_p3(S, t);
  ge_p3_to_cached(out, S);
}

// Positions the Straus loop must run for this wave: the largest need of its
// lanes (wave-uniform; 33 for almost every wave).  `need` in [1, 40].
STL_HD int half_positions(int need) {
#if defined(__HIP_DEVICE_COMPILE__)
  int p = 32;
#pragma unroll
  for (int b = 33; b <= kHalfDigits; ++b) p = __any(need >= b) ? b : p;
  return p;
#else
  return need > 32 ? need : 32;
#endif
}

// ---- wide base tables for [e]B ----
// Two tables of j*B and j*2^128*B, j = 0..32768 (entry 0 the identity), in
// affine Niels form (28 words, canonical limbs): e in signed radix 2^16 takes
// 16 mixed adds (8 per table, one at every fourth nibble position) instead of
// 32 with the 128-entry LDS tables.  7.3 MB per device, built once at init
// (wide_entry) and read through L2 / the Infinity Cache.
constexpr uint32_t kWideEntries = 32769;
constexpr uint32_t kWideRowWords = 28;
constexpr size_t kWideTableWords = 2ull * kWideEntries * kWideRowWords;

// Row j of wide table `which` from the first entry (1*P) of the 128-entry
// base table: [j]P by double-and-add, then affine and canonical.
STL_HD void wide_entry(uint32_t row[28], int which, uint32_t j, const uint32_t* btab) {
  ge_niels P;
  load_base_niels(P, btab + which * kBaseTableWords, 1);
  ge_p3 acc;
  ge_p2 acc2;
  ge_p1p1 t;
  ge_p3_0(acc);
  ge_p2_0(acc2);
  for (int bit = 15; bit >= 0; --bit) {
    ge_p2_dbl(t, acc2);
    ge_p1p1_to_p3(acc, t);
    if ((j >> bit) & 1u) {
      ge_madd(t, acc, P);
      ge_p1p1_to_p3(acc, t);
    }
    ge_p3_to_p2(acc2, acc);
  }
  if (j >> 16) {  // j = 65536 does not occur (j <= 32768); kept total for safety
    ge_p3_0(acc);
  }
  fe zi, x, y, ypx, ymx, xy, xy2d, c2d;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_add(ypx, y, x);
  fe_carry(ypx);
  fe_sub(ymx, y, x);
  fe_mul(xy, x, y);
  fe_const_2d(c2d);
  fe_mul(xy2d, xy, c2d);
  uint32_t w[8];
  fe canon[3];
  fe_tobytes(w, ypx);
  fe_frombytes(canon[0], w);
  fe_tobytes(w, ymx);
  fe_frombytes(canon[1], w);
  fe_tobytes(w, xy2d);
  fe_frombytes(canon[2], w);
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < 9; ++i) row[9 * k + i] = canon[k].v[i];
  row[27] = 0;
}

// Wide-table reader of the host build: rows straight from memory.
struct WideHost {
  const uint32_t* tab;  // kWideTableWords
  int d[2];
  STL_HD void prefetch(int d0, int d1) {
    d[0] = d0;
    d[1] = d1;
  }
  STL_HD void madd(ge_p1p1& t, const ge_p3& acc, int which) const {
    const int a = d[which] < 0 ? -d[which] : d[which];
    const uint32_t* row = tab + ((size_t)which * kWideEntries + (uint32_t)a) * kWideRowWords;
    ge_niels n;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      n.ypx.v[i] = row[i];
      n.ymx.v[i] = row[9 + i];
      n.xy2d.v[i] = row[18 + i];
    }
    ge_niels_cneg(n, d[which] < 0);
    ge_madd(t, acc, n);
  }
};

// Phase 2 of the half-size check: [e]B + [c](-A) + [d](-Q) == O.  Joint
// Straus over the nibble positions of c and d (two per-lane 9-entry tables),
// with e's 16 radix-2^16 digits added from the wide tables at every fourth
// position.  `Wide` reads table rows (WideHost here; the kernel's stages
// them in LDS by asynchronous loads issued before the doublings).
// With `keytabs` (STL_DEDUP_KEYS) a wave whose lanes all carry kHalfKeyed
// reads the A-table from the shared per-key tables instead of building it;
// with `widetabs` and kHalfKeyedWide on every lane it adds c's digits in pairs
// (16*d_{2j+1} + d_{2j} at position 2j) from the key's 137-entry table.
template <typename Wide>
STL_HD bool verify_phase2_half(const HalfState& p, const TableView& tab1, const TableView& tab2, Wide& wide,
                               const uint4* keytabs = nullptr, const uint4* widetabs = nullptr) {
  bool keyed = keytabs != nullptr && (p.tops & kHalfKeyed) != 0;
  bool kwide = keyed && widetabs != nullptr && (p.tops & kHalfKeyedWide) != 0;
#if defined(__HIP_DEVICE_COMPILE__)
  keyed = __all(keyed);  // wave-uniform: the table source and the build are per wave
  kwide = __all(kwide);
#endif
  kwide = kwide && keyed;
  const bool a_flip = keyed && (p.tops & kHalfCNeg) != 0;  // key table holds j*(-A); P1 = +A when c < 0
  const TableView t1 =
      kwide ? TableView::contiguous(const_cast<uint4*>(widetabs) + (size_t)p.pad * (kWideKeyEntries * 9))
            : keyed ? TableView::contiguous(const_cast<uint4*>(keytabs) + (size_t)p.pad * kTableQuadsPerKey) : tab1;
  {
    ge_p3 P;
    if (!keyed) {
      affine_to_p3(P, p.P1x, p.P1y);
      build_cached_table(tab1, P);
    }
    affine_to_p3(P, p.P2x, p.P2y);
    build_cached_table(tab2, P);
  }
  const int npos = half_positions((int)(p.tops & 0xffu));
  uint32_t cd[5], dd[5], ed[8];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    cd[i] = p.cdig[i];
    dd[i] = p.ddig[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) ed[i] = p.edig[i];
  ge_p3 acc;
  ge_p2 acc2;
  ge_p1p1 t;
  ge_p3_0(acc);
  ge_p2_0(acc2);
  uint32_t wc = 0, wd = 0, we0 = 0, we1 = 0;
  int cprev = 0;  // kwide: c's digit of the odd position above, added with the next even one
#pragma unroll 1
  for (int i = kHalfDigits - 1; i >= 0; --i) {
    if ((i & 7) == 7) {  // next 8 radix-16 digits of |c| and |d|
      wc = cd[4];
      wd = dd[4];
#pragma unroll
      for (int m = 4; m > 0; --m) {
        cd[m] = cd[m - 1];
        dd[m] = dd[m - 1];
      }
    }
    if ((i & 7) == 4 && i < 32) {  // next 2 radix-2^16 digits of e, low and high halves
      we0 = ed[3];
      we1 = ed[7];
#pragma unroll
      for (int m = 3; m > 0; --m) {
        ed[m] = ed[m - 1];
        ed[4 + m] = ed[4 + m - 1];
      }
    }
    int dc = (int32_t)wc >> 28;
    const int dq = (int32_t)wd >> 28;
    wc <<= 4;
    wd <<= 4;
    bool cadd = true;  // wave-uniform
    if (kwide) {
      if (i & 1) {
        cprev = dc;
        cadd = false;
      } else {
        dc += 16 * cprev;
        cprev = 0;
      }
    }
    const bool bpos = (i & 3) == 0 && i < 32;  // wave-uniform
    int de0 = 0, de1 = 0;
    if (bpos) {
      de0 = (i & 4) ? (int32_t)we0 >> 16 : (int32_t)(we0 << 16) >> 16;
      de1 = (i & 4) ? (int32_t)we1 >> 16 : (int32_t)(we1 << 16) >> 16;
    }
    if (i >= npos) continue;  // wave-uniform: digits above every lane's need are 0
    // Issue this position's table loads ahead of the doublings (~15k cycles
    // of independent work per wave): their latency (L2 / Infinity Cache) is
    // hidden instead of stalling the adds.
    ge_cached ca, cq;
    // Unconditional loads (entry 0 where a wide-key position skips the A-add):
    // a load under `if (cadd)` made the compiler merge its registers at the
    // end of the branch, i.e. wait for the load there -- before the doublings
    // it is meant to overlap.
    t1.load(cadd ? (dc < 0 ? -dc : dc) : 0, ca);
    tab2.load(dq < 0 ? -dq : dq, cq);
    if (bpos) wide.prefetch(de0, de1);
    if (i != npos - 1) dbl4(acc, acc2);
    if (cadd) {
      ge_cached_cneg(ca, (dc < 0) != a_flip);
      ge_add_cached(t, acc, ca);
      ge_p1p1_to_p3(acc, t);
    }
    ge_cached_cneg(cq, dq < 0);
    ge_add_cached(t, acc, cq);
    if (!bpos) {
      ge_p1p1_to_p2(acc2, t);
    } else {
      ge_p1p1_to_p3(acc, t);
      wide.madd(t, acc, 0);
      ge_p1p1_to_p3(acc, t);
      wide.madd(t, acc, 1);
      ge_p1p1_to_p2(acc2, t);
    }
  }
  // identity: X == 0 and Y == Z
  fe ymz;
  fe_sub(ymz, acc2.Y, acc2.Z);
  const bool id = fe_iszero(acc2.X) && fe_iszero(ymz);
  return (p.tops & kHalfOk) != 0 && (p.tops & kHalfFallback) == 0 && id;
}

// ---- joint radix-4 table (round 3): one per-lane table for both points ----
// c and d in signed radix 16 (digits D in [-8, 7]) are read as signed radix 4:
// D = 4q + r with r = ((D + 2) mod 4) - 2 in [-2, 1] and q in [-2, 2], so a
// nibble position becomes two sub-positions, each two doublings and ONE add
// of a*P1 + b*P2 with (a, b) in [-2, 2]^2 -- the same 4 doublings and 2 adds
// per nibble as two radix-16 tables, but the table holds 12 entries (the
// pairs up to sign) instead of 2 x 8, built with 36 products fewer, and the
// per-lane heads shrink from 2 KiB to 1.5 KiB.  Index of (a, b) up to sign:
//   (0, 1), (0, 2)                      -> 1, 2
//   (1, b), b = -2..2 / (2, b)          -> 3..7 / 8..12
// entry 0 is the identity (a = b = 0).
constexpr int kJointEntries = 12;

STL_HD int joint_index(int a, int b, bool& neg) {
  neg = a < 0 || (a == 0 && b < 0);
  if (neg) {
    a = -a;
    b = -b;
  }
  return a == 0 ? b : 3 + (a - 1) * 5 + (b + 2);
}

// -(cached point) with every limb normalised (T2d [1], so a lookup may negate
// it again with fe_neg_nc<2>)
STL_HD void ge_cached_neg_norm(ge_cached& c) {
  const fe a = c.YpX;
  c.YpX = c.YmX;
  c.YmX = a;
  fe_neg(c.T2d, c.T2d);
}

// p3 -> cached, stored at entry e
STL_HD void joint_store(const TableView& tab, int e, const ge_p3& P) {
  ge_cached c;
  ge_p3_to_cached(c, P);
  tab.store(e, c);
}

// 2P from a p3 point (a projective doubling), -> p3
STL_HD void ge_p3_dbl_p3(ge_p3& r, const ge_p3& P) {
  ge_p2 p2;
  ge_p1p1 t;
  ge_p3_to_p2(p2, P);
  ge_p2_dbl(t, p2);
  ge_p1p1_to_p3(r, t);
}

// Affine point i (0: P1, 1: P2) of a HalfState in memory (words 20-55).
STL_HD void state_point(ge_p3& P, const uint4* state, int i) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(state) + 20 + 18 * i;
  fe x, y;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    x.v[k] = w[k];
    y.v[k] = w[9 + k];
  }
  affine_to_p3(P, x, y);
}

// Niels form of a stored Z = 1 entry (P1 at 5, P2 at 1), sign applied.
STL_HD void joint_niels(ge_niels& n, const TableView& tab, int e, bool neg) {
  ge_cached c;
  tab.load(e, c);
  n.ypx = c.YpX;
  n.ymx = c.YmX;
  n.xy2d = c.T2d;
  ge_niels_cneg(n, neg);
}

// The 12 entries a*P1 + b*P2 from the affine P1, P2 of the lane's HalfState
// in memory: 72 M + 14 S against 108 M + 6 S for two 8-entry tables.  Points
// are re-read from the state and Niels forms from the entries already stored
// (L1 / L2 hits) rather than held, so at most two points and one Niels form
// are live next to the products' registers.
STL_HD void build_joint_table(const TableView& tab, const uint4* state) {
  ge_p1p1 t;
  {
    ge_cached c;
    ge_cached_0(c);
    tab.store(0, c);
    ge_p3 P2;
    state_point(P2, state, 1);
    joint_store(tab, 1, P2);  // (0, 1); Z = 1, so its cached form is its Niels form
    ge_affine_dbl(t, P2);
    ge_p1p1_to_p3(P2, t);
    joint_store(tab, 2, P2);  // (0, 2)
  }
  {
    ge_p3 P1, S;
    state_point(P1, state, 0);
    joint_store(tab, 5, P1);  // (1, 0)
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {  // P1 + P2, then P1 - P2, and their doubles
      ge_niels n;
      joint_niels(n, tab, 1, s == 1);
      ge_madd(t, P1, n);
      ge_p1p1_to_p3(S, t);
      joint_store(tab, s == 0 ? 6 : 4, S);  // (1, 1) / (1, -1)
      ge_p3_dbl_p3(S, S);
      joint_store(tab, s == 0 ? 12 : 8, S);  // (2, 2) / (2, -2)
    }
    ge_affine_dbl(t, P1);
    ge_p1p1_to_p3(P1, t);  // P1 <- 2 P1
    joint_store(tab, 10, P1);  // (2, 0)
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {  // 2 P1 + P2, 2 P1 - P2
      ge_niels n;
      joint_niels(n, tab, 1, s == 1);
      ge_madd(t, P1, n);
      ge_p1p1_to_p3(S, t);
      joint_store(tab, s == 0 ? 11 : 9, S);  // (2, 1) / (2, -1)
    }
  }
  {
    ge_p3 Q, S;
    state_point(Q, state, 1);
    ge_affine_dbl(t, Q);
    ge_p1p1_to_p3(Q, t);  // 2 P2 (recomputed: cheaper than holding it)
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {  // 2 P2 + P1 = (1, 2); 2 P2 - P1 = -(1, -2)
      ge_niels n;
      joint_niels(n, tab, 5, s == 1);
      ge_madd(t, Q, n);
      ge_p1p1_to_p3(S, t);
      ge_cached c;
      ge_p3_to_cached(c, S);
      if (s == 1) ge_cached_neg_norm(c);
      tab.store(s == 0 ? 7 : 3, c);
    }
  }
}

// Phase 2 with the joint table: [e]B + [c](-A) + [d](-Q) == O as in
// verify_phase2_half (same digits, same wide-table madds at every fourth
// nibble position, same identity test); one table, one add per sub-position.
// `state` is the lane's HalfState in memory (14 quads): the points are read
// for the table build, the digits and flags only after it, so they are not
// held in registers across the build.
template <typename Wide>
STL_HD bool verify_phase2_joint(const uint4* state, const TableView& tab, Wide& wide) {
  build_joint_table(tab, state);
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" ::: "memory");  // the digit loads stay after the build
#endif
  HalfState p;
  {
    uint32_t* w = reinterpret_cast<uint32_t*>(&p);
    const uint32_t* s = reinterpret_cast<const uint32_t*>(state);
#pragma unroll
    for (int i = 0; i < 20; ++i) w[i] = s[i];
  }
  const int npos = half_positions((int)(p.tops & 0xffu));
  uint32_t cd[5], dd[5], ed[8];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    cd[i] = p.cdig[i];
    dd[i] = p.ddig[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) ed[i] = p.edig[i];
  ge_p3 acc;
  ge_p2 acc2;
  ge_p1p1 t;
  ge_p3_0(acc);
  ge_p2_0(acc2);
  uint32_t wc = 0, wd = 0, we0 = 0, we1 = 0;
#pragma unroll 1
  for (int i = kHalfDigits - 1; i >= 0; --i) {
    if ((i & 7) == 7) {
      wc = cd[4];
      wd = dd[4];
#pragma unroll
      for (int m = 4; m > 0; --m) {
        cd[m] = cd[m - 1];
        dd[m] = dd[m - 1];
      }
    }
    if ((i & 7) == 4 && i < 32) {
      we0 = ed[3];
      we1 = ed[7];
#pragma unroll
      for (int m = 3; m > 0; --m) {
        ed[m] = ed[m - 1];
        ed[4 + m] = ed[4 + m - 1];
      }
    }
    const int dc = (int32_t)wc >> 28;
    const int dq = (int32_t)wd >> 28;
    wc <<= 4;
    wd <<= 4;
    const bool bpos = (i & 3) == 0 && i < 32;  // wave-uniform
    int de0 = 0, de1 = 0;
    if (bpos) {
      de0 = (i & 4) ? (int32_t)we0 >> 16 : (int32_t)(we0 << 16) >> 16;
      de1 = (i & 4) ? (int32_t)we1 >> 16 : (int32_t)(we1 << 16) >> 16;
    }
    if (i >= npos) continue;  // wave-uniform
    const int cr = ((dc + 2) & 3) - 2, dr = ((dq + 2) & 3) - 2;
    bool n0, n1;
    const int e0 = joint_index((dc - cr) >> 2, (dq - dr) >> 2, n0);
    const int e1 = joint_index(cr, dr, n1);
    if (bpos) wide.prefetch(de0, de1);
    // the two sub-positions share one copy of the code (the loop body stays
    // about the size of the two-table loop's): load the entry, two doublings
    // while it arrives, one addition
#pragma unroll 1
    for (int sub = 0; sub < 2; ++sub) {
      ge_cached c;
      tab.load(sub == 0 ? e0 : e1, c);
      if (sub == 1 || i != npos - 1) {
        ge_p2_dbl<true>(t, acc2);
        ge_p1p1_to_p2(acc2, t);
        ge_p2_dbl(t, acc2);
        ge_p1p1_to_p3(acc, t);
      }
      ge_cached_cneg(c, sub == 0 ? n0 : n1);
      ge_add_cached(t, acc, c);
      if (sub == 0 || !bpos) ge_p1p1_to_p2(acc2, t);
    }
    if (bpos) {
      ge_p1p1_to_p3(acc, t);
      wide.madd(t, acc, 0);
      ge_p1p1_to_p3(acc, t);
      wide.madd(t, acc, 1);
      ge_p1p1_to_p2(acc2, t);
    }
  }
  fe ymz;
  fe_sub(ymz, acc2.Y, acc2.Z);
  const bool id = fe_iszero(acc2.X) && fe_iszero(ymz);
  return (p.tops & kHalfOk) != 0 && (p.tops & kHalfFallback) == 0 && id;
}

// Small batches (at most a quarter of the resident lanes, launch_verify's
// pair_max: one pair wave per SIMD): one signature on two lanes.  Lane `par` = 0 runs [e_lo]B + [c]P1 (the low
// wide table), lane 1 runs [e_hi]2^128 B + [d]P2 (the high one), on the same
// doubling schedule as verify_phase2_half -- one table, one add per position
// and one madd per fourth position instead of two each.  The pair then checks
// that its two sums cancel (pair_sums_cancel).  Same accept bits; about 0.77x
// of a lane's chain, so a launch whose lanes are not all busy ends sooner.
template <typename Wide>
STL_HD void verify_phase2_pair_chain(ge_p2& out, const HalfState& p, int par, const TableView& tab, Wide& wide) {
  {
    ge_p3 P;
    affine_to_p3(P, par ? p.P2x : p.P1x, par ? p.P2y : p.P1y);
    build_cached_table(tab, P);
  }
  const int npos = half_positions((int)(p.tops & 0xffu));
  uint32_t dg[5], ed[4];
#pragma unroll
  for (int i = 0; i < 5; ++i) dg[i] = par ? p.ddig[i] : p.cdig[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) ed[i] = par ? p.edig[4 + i] : p.edig[i];
  ge_p3 acc;
  ge_p2 acc2;
  ge_p1p1 t;
  ge_p3_0(acc);
  ge_p2_0(acc2);
  uint32_t w = 0, we = 0;
#pragma unroll 1
  for (int i = kHalfDigits - 1; i >= 0; --i) {
    if ((i & 7) == 7) {
      w = dg[4];
#pragma unroll
      for (int m = 4; m > 0; --m) dg[m] = dg[m - 1];
    }
    if ((i & 7) == 4 && i < 32) {
      we = ed[3];
#pragma unroll
      for (int m = 3; m > 0; --m) ed[m] = ed[m - 1];
    }
    const int d = (int32_t)w >> 28;
    w <<= 4;
    const bool bpos = (i & 3) == 0 && i < 32;  // wave-uniform
    int de = 0;
    if (bpos) de = (i & 4) ? (int32_t)we >> 16 : (int32_t)(we << 16) >> 16;
    if (i >= npos) continue;  // wave-uniform
    ge_cached c;
    tab.load(d < 0 ? -d : d, c);  // issued ahead of the doublings, as in verify_phase2_half
    if (bpos) wide.prefetch(par ? 0 : de, par ? de : 0);
    if (i != npos - 1) dbl4(acc, acc2);
    ge_cached_cneg(c, d < 0);
    ge_add_cached(t, acc, c);
    if (!bpos) {
      ge_p1p1_to_p2(acc2, t);
    } else {
      ge_p1p1_to_p3(acc, t);
      wide.madd(t, acc, par);
      ge_p1p1_to_p2(acc2, t);
    }
  }
  out = acc2;
}

// a + b == O  <=>  a == -b  <=>  Xa Zb == -Xb Za and Ya Zb == Yb Za (Z != 0).
STL_HD bool pair_sums_cancel(const ge_p2& a, const ge_p2& b) {
  fe l, r, s;
  fe_mul(l, a.X, b.Z);
  fe_mul(r, b.X, a.Z);
  fe_add(s, l, r);
  fe_carry(s);
  const bool xs = fe_iszero(s);
  fe_mul(l, a.Y, b.Z);
  fe_mul(r, b.Y, a.Z);
  fe_sub(s, l, r);
  return xs && fe_iszero(s);
}

STL_HD bool half_state_accepts(const HalfState& p) {
  return (p.tops & kHalfOk) != 0 && (p.tops & kHalfFallback) == 0;
}


}  // namespace stl
