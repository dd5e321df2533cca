// Edwards25519 group arithmetic on top of fe25519.h (one point per lane).
//
// Coordinates (twisted Edwards, a = -1, d = -121665/121666):
//   ge_p2     (X:Y:Z)            x = X/Z, y = Y/Z
//   ge_p3     (X:Y:Z:T)          extended, T = XY/Z
//   ge_p1p1   (X:Y:Z:T)          "completed": x = X/Z, y = Y/T (output of add/dbl)
//   ge_cached (Y+X, Y-X, Z, 2dT) for the variable-base table
//   ge_niels  (y+x, y-x, 2dxy)   affine, for the fixed basepoint table
// Formulas: add-2008-hwcd-3 (unified addition) and dbl-2008-hwcd from the Explicit-Formulas
// Database; both are complete on Ed25519 because d is a non-square.  The results are group
// elements, so the verdicts are independent of the chosen formulas (dalek compares points,
// SURVEY.md A.3 step 5).
#pragma once
#include "fe25519.h"
#include "consts.h"

namespace nwc {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

FE_DEV ge_p3 ge_p3_identity() { ge_p3 r; r.X = fe_zero(); r.Y = fe_one(); r.Z = fe_one(); r.T = fe_zero(); return r; }
FE_DEV ge_cached ge_cached_identity() {
  ge_cached r; r.YpX = fe_one(); r.YmX = fe_one(); r.Z = fe_one(); r.T2d = fe_zero(); return r;
}
FE_DEV ge_niels ge_niels_identity() { ge_niels r; r.ypx = fe_one(); r.ymx = fe_one(); r.xy2d = fe_zero(); return r; }

FE_DEV ge_p2 ge_p1p1_to_p2(const ge_p1p1& p) {
  ge_p2 r; r.X = fe_mul(p.X, p.T); r.Y = fe_mul(p.Y, p.Z); r.Z = fe_mul(p.Z, p.T); return r;
}
FE_DEV ge_p3 ge_p1p1_to_p3(const ge_p1p1& p) {
  ge_p3 r; r.X = fe_mul(p.X, p.T); r.Y = fe_mul(p.Y, p.Z); r.Z = fe_mul(p.Z, p.T); r.T = fe_mul(p.X, p.Y); return r;
}
// The same conversions for a completed point whose Y is the sum of two tight elements (the output
// of ge_p2_dbl, of the cached/Niels additions, or of a re-centred table entry -- the ladders'
// accumulator): fe_mul(f, g) prepares 2 f_i (odd i) and 19 g_j once per distinct operand, so with
// Y on the right the four products share two f's (X, Z) and two g's (T, Y): 9 v_mul_lo_u32 and 5
// shifts fewer than (X.T, Y.Z, Z.T, X.Y).  Y as a right operand needs |19 Y_j| < 2^31, which a
// sum of two tight elements meets (2^30.3) and 2y from an unreduced Niels entry does not.
FE_DEV ge_p2 ge_p1p1_to_p2_acc(const ge_p1p1& p) {
  ge_p2 r; r.X = fe_mul(p.X, p.T); r.Y = fe_mul(p.Z, p.Y); r.Z = fe_mul(p.Z, p.T); return r;
}
FE_DEV ge_p3 ge_p1p1_to_p3_acc(const ge_p1p1& p) {
  ge_p3 r; r.X = fe_mul(p.X, p.T); r.Y = fe_mul(p.Z, p.Y); r.Z = fe_mul(p.Z, p.T); r.T = fe_mul(p.X, p.Y); return r;
}
FE_DEV ge_p2 ge_p3_to_p2(const ge_p3& p) { ge_p2 r; r.X = p.X; r.Y = p.Y; r.Z = p.Z; return r; }
FE_DEV ge_cached ge_p3_to_cached(const ge_p3& p) {
  ge_cached r; r.YpX = fe_add(p.Y, p.X); r.YmX = fe_sub(p.Y, p.X); r.Z = p.Z; r.T2d = fe_mul(p.T, FE_D2); return r;
}
FE_DEV ge_p3 ge_p3_neg(const ge_p3& p) { ge_p3 r = p; r.X = fe_neg(p.X); r.T = fe_neg(p.T); return r; }

// dbl-2008-hwcd, a = -1: from (X:Y:Z) only (T not needed).  4 squarings.
FE_DEV ge_p1p1 ge_p2_dbl(const ge_p2& p) {
  ge_p1p1 r;
  fe xx = fe_sq(p.X);
  fe yy = fe_sq(p.Y);
  fe b = fe_sq2(p.Z);
  fe a = fe_sq(fe_add(p.X, p.Y));
  r.Y = fe_add(yy, xx);          // -H
  r.Z = fe_sub(yy, xx);          //  G
  r.X = fe_sub(a, r.Y);          //  E
  r.T = fe_sub(b, r.Z);          // -F
  return r;
}

// p + q, q cached.  4 multiplications.
FE_DEV ge_p1p1 ge_add_cached(const ge_p3& p, const ge_cached& q) {
  ge_p1p1 r;
  fe pp = fe_mul(fe_add(p.Y, p.X), q.YpX);
  fe mm = fe_mul(fe_sub(p.Y, p.X), q.YmX);
  fe tt = fe_mul(p.T, q.T2d);
  fe zz = fe_mul(p.Z, q.Z);
  fe zz2 = fe_add(zz, zz);
  r.X = fe_sub(pp, mm);
  r.Y = fe_add(pp, mm);
  r.Z = fe_add(zz2, tt);
  r.T = fe_sub(zz2, tt);
  return r;
}

// p + q, q affine niels.  3 multiplications.
FE_DEV ge_p1p1 ge_add_niels(const ge_p3& p, const ge_niels& q) {
  ge_p1p1 r;
  fe pp = fe_mul(fe_add(p.Y, p.X), q.ypx);
  fe mm = fe_mul(fe_sub(p.Y, p.X), q.ymx);
  fe tt = fe_mul(p.T, q.xy2d);
  fe zz2 = fe_add(p.Z, p.Z);
  r.X = fe_sub(pp, mm);
  r.Y = fe_add(pp, mm);
  r.Z = fe_add(zz2, tt);
  r.T = fe_sub(zz2, tt);
  return r;
}

// Conditional negation of a table entry: -(x, y) = (-x, y) swaps Y+X <-> Y-X and negates T.
FE_DEV ge_cached ge_cached_cneg(const ge_cached& q, bool neg) {
  ge_cached r;
  r.YpX = fe_select(q.YpX, q.YmX, neg);
  r.YmX = fe_select(q.YmX, q.YpX, neg);
  r.Z = q.Z;
  r.T2d = fe_select(q.T2d, fe_neg(q.T2d), neg);
  return r;
}
FE_DEV ge_niels ge_niels_cneg(const ge_niels& q, bool neg) {
  ge_niels r;
  r.ypx = fe_select(q.ypx, q.ymx, neg);
  r.ymx = fe_select(q.ymx, q.ypx, neg);
  r.xy2d = fe_select(q.xy2d, fe_neg(q.xy2d), neg);
  return r;
}

// curve25519-dalek CompressedEdwardsY::decompress of N (1 or 2) encodings at once:
//   y = low 255 bits (y >= p accepted), u = y^2 - 1, v = d y^2 + 1, (ok, x) = sqrt_ratio_i(u, v),
//   x := -x if the sign bit is set -- even when x == 0.
// The two 252-squaring exponentiations are serial chains; running A's and R's side by side gives
// the scheduler two independent chains per lane.  Also returns the canonical y words (for the
// small-order test).
// Before the exponentiation: y, u = y^2 - 1, v^3 and z = u v^7 (v = d y^2 + 1).
FE_DEV void ge_decompress_prep(const u32* w, fe& y, fe& u, fe& v3, fe& z) {
  const fe one = fe_one();
  y = fe_from_words(w);
  const fe yy = fe_sq(y);
  u = fe_sub(yy, one);
  const fe v = fe_add(fe_mul(yy, FE_D), one);
  v3 = fe_mul(fe_sq(v), v);
  const fe v7 = fe_mul(fe_sq(v3), v);
  z = fe_mul(u, v7);
}
// After it (b = z^((p-5)/8)): r = u v^3 b, the sqrt_ratio_i checks, sign fix-ups, the point.
FE_DEV void ge_decompress_finish(const u32* w, const fe& y, const fe& u, const fe& v3, const fe& b, ge_p3& out,
                                 u32 ycanon[8], bool& ok) {
  const fe one = fe_one();
  // r = u v^3 (u v^7)^((p-5)/8); check = v r^2
  fe r = fe_mul(fe_mul(u, v3), b);
  const fe yy = fe_sq(y);
  const fe vv = fe_add(fe_mul(yy, FE_D), one);
  fe check = fe_mul(vv, fe_sq(r));
  const bool correct = fe_equal(check, u);
  const bool flipped = fe_is_zero(fe_add(check, u));
  const bool flipped_i = fe_is_zero(fe_add(check, fe_mul(u, FE_SQRTM1)));
  r = fe_select(r, fe_mul(r, FE_SQRTM1), flipped || flipped_i);
  r = fe_select(r, fe_neg(r), fe_is_negative(r));
  const bool sign = (w[7] >> 31) & 1;
  const fe x = fe_select(r, fe_neg(r), sign);
  const fe yt = fe_tighten(y);
  out.X = x;
  out.Y = yt;
  out.Z = one;
  out.T = fe_mul(x, yt);
  fe_to_words(y, ycanon);
  ok = correct || flipped;
}

template <int N>
FE_DEV void ge_decompressN(ge_p3 out[N], const u32* const w[N], u32 ycanon[N][8], bool ok[N]) {
  fe y[N], u[N], v[N], z[N];
  _Pragma("unroll") for (int k = 0; k < N; ++k) ge_decompress_prep(w[k], y[k], u[k], v[k], z[k]);
  // z^(2^252 - 3) for both, interleaved
  fe a[N], b[N], t[N];
#define BOTH(stmt) _Pragma("unroll") for (int k = 0; k < N; ++k) { stmt; }
  fe z2[N], z9[N], z11[N];
  BOTH(z2[k] = fe_sq(z[k]));
  BOTH(t[k] = fe_sq(fe_sq(z2[k])));
  BOTH(z9[k] = fe_mul(z[k], t[k]));
  BOTH(z11[k] = fe_mul(z2[k], z9[k]));
  BOTH(a[k] = fe_mul(z9[k], fe_sq(z11[k])));                 // 2^5 - 1
  fe t10[N], t50[N];
  BOTH(t[k] = a[k]);
  _Pragma("unroll 1") for (int i = 0; i < 5; ++i) BOTH(t[k] = fe_sq(t[k]));
  BOTH(t10[k] = fe_mul(t[k], a[k]));                         // 2^10 - 1
  BOTH(t[k] = t10[k]);
  _Pragma("unroll 1") for (int i = 0; i < 10; ++i) BOTH(t[k] = fe_sq(t[k]));
  BOTH(b[k] = fe_mul(t[k], t10[k]));                         // 2^20 - 1
  BOTH(t[k] = b[k]);
  _Pragma("unroll 1") for (int i = 0; i < 20; ++i) BOTH(t[k] = fe_sq(t[k]));
  BOTH(b[k] = fe_mul(t[k], b[k]));                           // 2^40 - 1
  _Pragma("unroll 1") for (int i = 0; i < 10; ++i) BOTH(b[k] = fe_sq(b[k]));
  BOTH(t50[k] = fe_mul(b[k], t10[k]));                       // 2^50 - 1
  BOTH(t[k] = t50[k]);
  _Pragma("unroll 1") for (int i = 0; i < 50; ++i) BOTH(t[k] = fe_sq(t[k]));
  BOTH(b[k] = fe_mul(t[k], t50[k]));                         // 2^100 - 1
  BOTH(t[k] = b[k]);
  _Pragma("unroll 1") for (int i = 0; i < 100; ++i) BOTH(t[k] = fe_sq(t[k]));
  BOTH(b[k] = fe_mul(t[k], b[k]));                           // 2^200 - 1
  _Pragma("unroll 1") for (int i = 0; i < 50; ++i) BOTH(b[k] = fe_sq(b[k]));
  BOTH(b[k] = fe_mul(b[k], t50[k]));                         // 2^250 - 1
  BOTH(b[k] = fe_mul(fe_sq(fe_sq(b[k])), z[k]));             // 2^252 - 3
#undef BOTH
  _Pragma("unroll") for (int k = 0; k < N; ++k) ge_decompress_finish(w[k], y[k], u[k], v[k], b[k], out[k], ycanon[k], ok[k]);
}

// One encoding, no pointer indirection (for inlined call sites whose input words live in VGPRs).
FE_DEV void ge_decompress1(const u32 w[8], ge_p3& out, u32 ycanon[8], bool& ok) {
  fe y, u, v3, z;
  ge_decompress_prep(w, y, u, v3, z);
  const fe b = fe_pow22523(z);
  ge_decompress_finish(w, y, u, v3, b, out, ycanon, ok);
}

// A decompressed point is small-order iff its y is one of the five y-coordinates of E[8]
// (0, 1, -1, +-y8): every such y decodes, and E[8] has exactly these y values.  Equivalent
// to dalek's `mul_by_cofactor().is_identity()` for decoded points.
FE_DEV bool ycanon_is_small_order(const u32 y[8]) {
  bool so = false;
  _Pragma("unroll") for (int k = 0; k < 5; ++k) {
    u32 diff = 0;
    _Pragma("unroll") for (int i = 0; i < 8; ++i) diff |= y[i] ^ SMALL_ORDER_Y[k][i];
    so = so || (diff == 0);
  }
  return so;
}

}  // namespace nwc
