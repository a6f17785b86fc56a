// stl_ge25519.h -- edwards25519 group operations (a = -1 twisted Edwards,
// extended coordinates), in the representations ref10 uses:
//   p2 (X:Y:Z), p3 (X:Y:Z:T), p1p1 ((X:Z),(Y:T)), cached (Y+X, Y-X, Z, 2dT),
//   niels (y+x, y-x, 2dxy) for affine table points.
// Limb bounds (see stl_fe25519.h) are annotated as [alpha].
#pragma once
#include "stl_fe25519.h"

namespace stl {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

// Products interleaved per group formula: 4 (default; 3-4 independent mad
// chains per wave, for 2 waves/SIMD) or 2 (fewer live registers, for kernels
// that run more waves per SIMD).
#ifndef STL_GE_NOPS
#define STL_GE_NOPS 4
#endif

STL_HD void ge_p2_0(ge_p2& h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); }
STL_HD void ge_p3_0(ge_p3& h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); fe_0(h.T); }
STL_HD void ge_cached_0(ge_cached& h) { fe_1(h.YpX); fe_1(h.YmX); fe_1(h.Z); fe_0(h.T2d); }

// p1p1 inputs (from dbl / add / madd below) have X [<=3], Y [<=2], Z [<=3],
// T [1]: X*T <= 3, Y*Z <= 6, Z*T <= 3, X*Y <= 6 (fe_mul needs <= 7).
STL_HD void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe X, Y, Z;
  fe_mul3(X, p.X, p.T, Y, p.Y, p.Z, Z, p.Z, p.T);
  r.X = X;
  r.Y = Y;
  r.Z = Z;
}

STL_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe X, Y, Z, T;
  fe_mul4(X, p.X, p.T, Y, p.Y, p.Z, Z, p.Z, p.T, T, p.X, p.Y);
  r.X = X;
  r.Y = Y;
  r.Z = Z;
  r.T = T;
}

STL_HD void ge_p3_to_p2(ge_p2& r, const ge_p3& p) { r.X = p.X; r.Y = p.Y; r.Z = p.Z; }

// Table entries are stored normalised [1].
STL_HD void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  fe_add(r.YpX, p.Y, p.X);
  fe_carry(r.YpX);
  fe_sub(r.YmX, p.Y, p.X);
  r.Z = p.Z;
  fe c2d;
  fe_const_2d(c2d);
  fe_mul(r.T2d, p.T, c2d);
}

// dbl-2008-hwcd (a = -1): p2 [1] -> p1p1 with X,T [1], Y [2], Z [3].
// TO_P2: the result only feeds ge_p1p1_to_p2 (X*T, Y*Z, Z*T; no X*Y), so X
// may stay lazy: X = A + 3*Z1 - Y [<= 4] (Y [<= 2+2^-11] < 3), X*T <= 4.
template <bool TO_P2 = false>
STL_HD void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe XX, YY, ZZ2, A, XpY;
  fe_add(XpY, p.X, p.Y);     // [2]
  fe_sq4(XX, p.X, YY, p.Y, ZZ2, p.Z, A, XpY);  // A [1]  (2^2 <= 7)
  fe_add(ZZ2, ZZ2, ZZ2);     // [2]
  fe_add(r.Y, YY, XX);       // [2]
  fe_sub_nc<2>(r.Z, YY, XX); // [3]
  if (TO_P2)
    fe_sub_nc<3>(r.X, A, r.Y);  // [4]
  else
    fe_sub(r.X, A, r.Y);     // [1]
  fe_sub(r.T, ZZ2, r.Z);     // [1]
}

// ge_p2_dbl for an affine point (Z = 1): 2 Z^2 = 2, three squarings instead
// of four; same output bounds.
STL_HD void ge_affine_dbl(ge_p1p1& r, const ge_p3& p) {
  fe XX, YY, ZZ2, A, XpY;
  fe_add(XpY, p.X, p.Y);     // [2]
  {
    const fe* a[3] = {&p.X, &p.Y, &XpY};
    fe h[3];
    fe_sq_n<3>(h, a);
    XX = h[0];
    YY = h[1];
    A = h[2];                // [1]  (2^2 <= 7)
  }
  fe_0(ZZ2);
  ZZ2.v[0] = 2;              // 2 Z^2
  fe_add(r.Y, YY, XX);       // [2]
  fe_sub_nc<2>(r.Z, YY, XX); // [3]
  fe_sub(r.X, A, r.Y);       // [1]
  fe_sub(r.T, ZZ2, r.Z);     // [1]
}

// add-2008-hwcd-3: p3 [1] + cached [1; T2d <= 2] -> p1p1 with X [3], Y [2],
// Z [3], T [1].
STL_HD void ge_add_cached(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe A, B, C, D, t, t2;
  fe_sub_nc<2>(t, p.Y, p.X); // [3]
  fe_add(t2, p.Y, p.X);      // [2]
  fe_mul4(A, t, q.YmX, B, t2, q.YpX, C, q.T2d, p.T, D, p.Z, q.Z);  // 3*1, 2*1, 2*1, 1*1
  fe_add(D, D, D);           // [2]
  fe_sub_nc<2>(r.X, B, A);   // [3]
  fe_add(r.Y, B, A);         // [2]
  fe_add(r.Z, D, C);         // [3]
  fe_sub(r.T, D, C);         // [1]
}

// madd: p3 [1] + niels [1; xy2d <= 2] (Z2 = 1) -> p1p1 with X [3], Y [2],
// Z [3], T [1].
STL_HD void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe A, B, C, D, t, t2;
  fe_sub_nc<2>(t, p.Y, p.X); // [3]
  fe_add(t2, p.Y, p.X);      // [2]
  fe_mul3(A, t, q.ymx, B, t2, q.ypx, C, q.xy2d, p.T);
  fe_add(D, p.Z, p.Z);       // [2]
  fe_sub_nc<2>(r.X, B, A);   // [3]
  fe_add(r.Y, B, A);         // [2]
  fe_add(r.Z, D, C);         // [3]
  fe_sub(r.T, D, C);         // [1]
}

// Conditionally negate a cached point: -(Y+X, Y-X, Z, 2dT) = (Y-X, Y+X, Z, -2dT)
STL_HD void ge_cached_cneg(ge_cached& q, bool neg) {
  fe nt;
  fe_neg_nc<2>(nt, q.T2d);   // [2]
  fe a = q.YpX, b = q.YmX;
  fe_cmov(q.YpX, a, b, neg);
  fe_cmov(q.YmX, b, a, neg);
  fe_cmov(q.T2d, q.T2d, nt, neg);
}

STL_HD void ge_niels_cneg(ge_niels& q, bool neg) {
  fe nt;
  fe_neg_nc<2>(nt, q.xy2d);  // [2]
  fe a = q.ypx, b = q.ymx;
  fe_cmov(q.ypx, a, b, neg);
  fe_cmov(q.ymx, b, a, neg);
  fe_cmov(q.xy2d, q.xy2d, nt, neg);
}

// ge25519_frombytes_negate_vartime (libsodium 1.0.18 / ref10): decode the
// 32-byte encoding s and return -A.  ok = false when (y^2-1)/(dy^2+1) has no
// square root.  x == 0 with the sign bit set is accepted (libsodium does not
// reject it).  Branch-free: both root candidates are computed and selected.
STL_HD bool ge_frombytes_negate_vartime(ge_p3& h, const uint32_t s[8]) {
  fe u, v, v3, vxx, chk, one, d, sqm1, xs;
  fe_frombytes(h.Y, s);
  fe_1(h.Z);
  fe_1(one);
  fe_const_d(d);
  fe_sq(u, h.Y);
  fe_mul(v, u, d);
  fe_sub(u, u, one);         // u = y^2 - 1
  fe_add(v, v, one);         // v = d y^2 + 1
  fe_sq(v3, v);
  fe_mul(v3, v3, v);         // v^3
  fe_sq(h.X, v3);
  fe_mul(h.X, h.X, v);
  fe_mul(h.X, h.X, u);       // u v^7
  fe_pow22523(h.X, h.X);
  fe_mul(h.X, h.X, v3);
  fe_mul(h.X, h.X, u);       // x = u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, h.X);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);
  const bool m_ok = fe_iszero(chk);
  fe_add(chk, vxx, u);
  fe_carry(chk);
  const bool p_ok = fe_iszero(chk);
  fe_const_sqrtm1(sqm1);
  fe_mul(xs, h.X, sqm1);
  fe_cmov(h.X, h.X, xs, !m_ok);
  const uint32_t sign = s[7] >> 31;
  fe nx;
  fe_neg(nx, h.X);
  fe_cmov(h.X, h.X, nx, fe_isnegative(h.X) == sign);
  fe_mul(h.T, h.X, h.Y);
  return m_ok || p_ok;
}

// ge25519_tobytes: canonical y with the sign of x in bit 255.
STL_HD void ge_tobytes(uint32_t s[8], const ge_p2& h) {
  fe recip, x, y;
  fe_invert(recip, h.Z);
  fe_mul(x, h.X, recip);
  fe_mul(y, h.Y, recip);
  fe_tobytes(s, y);
  s[7] ^= fe_isnegative(x) << 31;
}

}  // namespace stl
