// Limb-sliced Edwards25519 group operations for latency-bound chains (gfx950), on top of
// fe_sliced.h.  A point's coordinates are `fes` values replicated over the four 16-lane rows of a
// wave; a *layer* assembles four operand pairs by row, runs ONE fes_mul for four independent
// products (row r computes product r), and re-broadcasts the four results to every row with
// v_permlane16_swap + 2 x v_permlane32_swap.  A doubling or an addition is two layers, so a
// serial point chain (the torsion test l*A of a first-sight key) runs ~2 x 78 instructions deep
// per step instead of ~1,000 with one point per lane.  Formulas and bounds are ge25519.h's
// (dbl-2008-hwcd, add-2008-hwcd-3); the doubling's 2 Z^2 takes its 2 on row 2's g operand, which
// stays inside fes_mul's int32 bound for a tight Z (|19 * 2 Z_i| < 2^31).
#pragma once
#include "fe_sliced.h"
#include "ge25519.h"

namespace nwc {

FES_DEV int fes_row() { return (int)((threadIdx.x >> 4) & 3); }

// row r <- a_r
FES_DEV fes fes_rows(fes a0, fes a1, fes a2, fes a3) {
  const int r = fes_row();
  const i32 lo = (r & 1) ? a1.v : a0.v, hi = (r & 1) ? a3.v : a2.v;
  return {(r & 2) ? hi : lo};
}

// out[r] = row r of x, on every row.  v_permlane16_swap(x, x) gives (x0, x0, x2, x2) and
// (x1, x1, x3, x3); v_permlane32_swap of each gives the four broadcasts.
FES_DEV void fes_bcast4(fes x, fes out[4]) {
  const auto p = __builtin_amdgcn_permlane16_swap((u32)x.v, (u32)x.v, false, false);
  const auto q = __builtin_amdgcn_permlane32_swap(p[0], p[0], false, false);
  const auto s = __builtin_amdgcn_permlane32_swap(p[1], p[1], false, false);
  out[0].v = (i32)q[0];
  out[1].v = (i32)s[0];
  out[2].v = (i32)q[1];
  out[3].v = (i32)s[1];
}

// one layer: out[r] = f_r * g_r for r = 0..3, replicated
FES_DEV void fes_mul4(fes f0, fes f1, fes f2, fes f3, fes g0, fes g1, fes g2, fes g3, fes out[4]) {
  fes_bcast4(fes_mul(fes_rows(f0, f1, f2, f3), fes_rows(g0, g1, g2, g3)), out);
}

struct gs_p2 { fes X, Y, Z; };
struct gs_p3 { fes X, Y, Z, T; };
struct gs_p1p1 { fes X, Y, Z, T; };
struct gs_cached { fes YpX, YmX, Z, T2d; };

// ge_p2_dbl: XX, YY, 2 Z^2, (X + Y)^2 in one layer
FES_DEV gs_p1p1 gs_dbl(const gs_p2& p) {
  const fes s = fes_add(p.X, p.Y);
  const fes z2 = fes_add(p.Z, p.Z);
  fes o[4];
  fes_mul4(p.X, p.Y, p.Z, s, p.X, p.Y, z2, s, o);
  gs_p1p1 r;
  r.Y = fes_add(o[1], o[0]);
  r.Z = fes_sub(o[1], o[0]);
  r.X = fes_sub(o[3], r.Y);
  r.T = fes_sub(o[2], r.Z);
  return r;
}
// completed -> projective / extended: X T, Y Z, Z T (, X Y) in one layer
FES_DEV gs_p2 gs_to_p2(const gs_p1p1& t) {
  fes o[4];
  fes_mul4(t.X, t.Y, t.Z, t.X, t.T, t.Z, t.T, t.Y, o);
  return {o[0], o[1], o[2]};
}
FES_DEV gs_p3 gs_to_p3(const gs_p1p1& t) {
  fes o[4];
  fes_mul4(t.X, t.Y, t.Z, t.X, t.T, t.Z, t.T, t.Y, o);
  return {o[0], o[1], o[2], o[3]};
}
// ge_add_cached: (Y+X)(Y2+X2), (Y-X)(Y2-X2), T T2d, Z Z2 in one layer
FES_DEV gs_p1p1 gs_add_cached(const gs_p3& p, const gs_cached& q) {
  const fes a = fes_add(p.Y, p.X), b = fes_sub(p.Y, p.X);
  fes o[4];
  fes_mul4(a, b, p.T, p.Z, q.YpX, q.YmX, q.T2d, q.Z, o);
  const fes zz2 = fes_add(o[3], o[3]);
  gs_p1p1 r;
  r.X = fes_sub(o[0], o[1]);
  r.Y = fes_add(o[0], o[1]);
  r.Z = fes_add(zz2, o[2]);
  r.T = fes_sub(zz2, o[2]);
  return r;
}
FES_DEV gs_cached gs_to_cached(const gs_p3& p) {
  gs_cached c;
  c.YpX = fes_add(p.Y, p.X);
  c.YmX = fes_sub(p.Y, p.X);
  c.Z = p.Z;
  c.T2d = fes_mul(p.T, fes_from_fe(FE_D2));
  return c;
}
FES_DEV gs_p2 gs_p3_to_p2(const gs_p3& p) { return {p.X, p.Y, p.Z}; }
// an affine point (x, y) held one element per lane -> extended, replicated over the rows
FES_DEV gs_p3 gs_from_affine(const fe& x, const fe& y) {
  gs_p3 r;
  r.X = fes_from_fe(x);
  r.Y = fes_from_fe(y);
  r.Z = fes_from_fe(fe_one());
  r.T = fes_mul(r.X, r.Y);
  return r;
}
FES_DEV bool gs_is_identity(const gs_p2& p) {
  return fe_is_zero(fe_from_fes(p.X)) && fe_is_zero(fe_from_fes(fes_sub(p.Y, p.Z)));
}

// [2^n] P from P's Edwards y alone: Montgomery u = (1 + y) / (1 - y) (Curve25519's birational
// map; the sign of x drops out), RFC 7748's x-only doubling (t1 = (U + W)^2, t2 = (U - W)^2,
// U' = t1 t2, W' = (t1 - t2)(t2 + 121666 (t1 - t2))), two layers per doubling.  Projective
// (U : W); the identity is (U : 0).  No square root: it can start before P is decompressed.
// y must be tight (fe_tighten): U - W = 2y feeds fes_mul, whose odd-limb bound 2y exceeds for
// raw fe_from_words limbs (tools/microbench/sliced_points.hip checks both against the doublings).
FES_DEV void gs_xonly_dbl_n(fes y, int n, fes& U, fes& W) {
  U = fes_add_small(y, 1);
  W = fes_add_small(fes_neg(y), 1);
#pragma unroll 1
  for (int k = 0; k < n; ++k) {
    const fes s = fes_add(U, W), d = fes_sub(U, W);
    fes t[4];
    fes_mul4(s, d, s, d, s, d, s, d, t);
    const fes e = fes_sub(t[0], t[1]);
    const fes g = fes_add(t[1], fes_mul_small(e, 121666));
    fes o[4];
    fes_mul4(t[0], e, t[0], e, t[1], g, t[1], g, o);
    U = o[0];
    W = o[1];
  }
}

// l * P != O (ge_has_torsion's double-and-add over l = 2^252 + c0, 252 doublings and 61 cached
// additions, every step limb-sliced)
FES_DEV bool gs_has_torsion(const gs_p3& P, const u32 l_words[8]) {
  const gs_cached pc = gs_to_cached(P);
  gs_p2 acc = gs_p3_to_p2(P);   // bit 252
#pragma unroll 1
  for (int bit = 251; bit >= 0; --bit) {
    gs_p1p1 t = gs_dbl(acc);
    if ((l_words[bit >> 5] >> (bit & 31)) & 1u) t = gs_add_cached(gs_to_p3(t), pc);
    acc = gs_to_p2(t);
  }
  return !gs_is_identity(acc);
}

}  // namespace nwc
