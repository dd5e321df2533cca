// Limb-sliced GF(2^255 - 19) arithmetic for latency-bound chains (gfx950).
//
// A field element is spread over one DPP row of 16 lanes: lane k (k = lane & 15) holds limb k of
// the radix-2^25.5 representation of fe25519.h for k < 10 and 0 for k >= 10, so a wave carries
// four independent elements (one per row) in ONE VGPR.  A product then costs one dependent chain
// of ~60 instructions instead of ~150 (fe_mul) / ~120 (fe_sq) in one lane: lane k accumulates
// column k itself,
//     h_k = sum_i f_i * g_(k-i mod 10) * [19 if i > k] * [2 if i and k-i are odd],
// with f_i broadcast across the row (DPP row_newbcast:i), g_(k-i) brought in by row_shr:i and the
// wrapped 19 g_(k-i+10) by row_shl:(10-i) from lanes that hold zero past limb 9.  Used where one
// element's dependent chain is the critical path (a square root inside the latency kernel); the
// throughput kernels keep one element per lane.
//
// Bounds are those of fe25519.h (inputs "loose", outputs "tight" + a small carry-in): the
// wrapped factor 19 goes on g (|19 g| < 2^31), the odd-odd factor 2 on g's odd limbs
// (|38 g_odd| < 2^31 for |g_odd| <= 1.65 * 2^25), column sums stay below 2^62.
#pragma once
#include "fe25519.h"

namespace nwc {

struct fes { i32 v; };

#define FES_DEV __device__ __forceinline__

FES_DEV int fes_lane() { return (int)(threadIdx.x & 15); }

// DPP row controls (gfx9): row_shl:n = 0x100 + n, row_shr:n = 0x110 + n, row_newbcast:n = 0x150 + n
template <int CTRL> FES_DEV i32 dpp(i32 x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true); }
template <int N> FES_DEV i32 row_shr(i32 x) { if constexpr (N == 0) return x; else return dpp<0x110 + N>(x); }
template <int N> FES_DEV i32 row_shl(i32 x) { if constexpr (N >= 16) return 0; else return dpp<0x100 + N>(x); }
template <int N> FES_DEV i32 row_bcast(i32 x) { return dpp<0x150 + N>(x); }

// one element per lane <-> one element per row (every row gets the same element)
FES_DEV fes fes_from_fe(const fe& a) {
  const int k = fes_lane();
  i32 r = 0;
  _Pragma("unroll") for (int i = 0; i < 10; ++i) r = k == i ? a.v[i] : r;
  return {r};
}
FES_DEV fe fe_from_fes(fes a) {
  fe r;
  r.v[0] = row_bcast<0>(a.v); r.v[1] = row_bcast<1>(a.v); r.v[2] = row_bcast<2>(a.v);
  r.v[3] = row_bcast<3>(a.v); r.v[4] = row_bcast<4>(a.v); r.v[5] = row_bcast<5>(a.v);
  r.v[6] = row_bcast<6>(a.v); r.v[7] = row_bcast<7>(a.v); r.v[8] = row_bcast<8>(a.v);
  r.v[9] = row_bcast<9>(a.v);
  return r;
}

// Products of term i: f_i (broadcast) times g_(k-i) or the wrapped 19 g_(k-i+10).  For odd i the
// odd-odd factor 2 is taken from the doubled-odd-limb copies gd / g19d.
template <int I>
FES_DEV void fes_term(i32 f, i32 g, i32 g19, i32 gd, i32 g19d, i64& acc) {
  const i32 b = row_bcast<I>(f);
  const i32 gs = (I & 1) ? gd : g, g19s = (I & 1) ? g19d : g19;
  const i32 s = row_shr<I>(gs) | row_shl<10 - I>(g19s);   // disjoint: one of them is 0 on every lane
  acc += (i64)b * (i64)s;
}

FES_DEV fes fes_mul(fes f, fes g) {
  const int k = fes_lane();
  const bool odd = (k & 1) != 0, live = k < 10;
  const i32 gl = live ? g.v : 0;   // lanes past limb 9 must read as zero
  const i32 g19 = (i32)(19u * (u32)gl);
  const i32 gd = odd ? (i32)((u32)gl << 1) : gl;
  const i32 g19d = odd ? (i32)((u32)g19 << 1) : g19;
  const int w = odd ? 25 : 26;
  i64 a0 = (i64)1 << (w - 1), a1 = 0;   // rounding bias on the column (fe25519.h fe_col_bias)
  fes_term<0>(f.v, gl, g19, gd, g19d, a0);
  fes_term<1>(f.v, gl, g19, gd, g19d, a1);
  fes_term<2>(f.v, gl, g19, gd, g19d, a0);
  fes_term<3>(f.v, gl, g19, gd, g19d, a1);
  fes_term<4>(f.v, gl, g19, gd, g19d, a0);
  fes_term<5>(f.v, gl, g19, gd, g19d, a1);
  fes_term<6>(f.v, gl, g19, gd, g19d, a0);
  fes_term<7>(f.v, gl, g19, gd, g19d, a1);
  fes_term<8>(f.v, gl, g19, gd, g19d, a0);
  fes_term<9>(f.v, gl, g19, gd, g19d, a1);
  const i64 h = a0 + a1;
  // round 1: column k's carry (up to 2^37) moves to column k + 1 (column 9's to column 0 x 19)
  const i64 c = h >> w;
  const u32 r = (u32)h & ((1u << w) - 1u);
  const i64 c19 = k == 9 ? c * 19 : 0;
  const i32 clo = row_shr<1>((i32)(u32)c) | row_shl<9>((i32)(u32)c19);
  const i32 chi = row_shr<1>((i32)(c >> 32)) | row_shl<9>((i32)(c19 >> 32));
  const i64 h2 = (i64)r + (i64)(((u64)(u32)chi << 32) | (u32)clo);
  // round 2: carries of at most 2^12 (x 19 into limb 0), limbs centred by removing the bias
  const i32 c2 = (i32)(h2 >> w);
  const u32 r2 = (u32)h2 & ((1u << w) - 1u);
  const i32 c219 = k == 9 ? c2 * 19 : 0;
  const i32 cin = row_shr<1>(c2) | row_shl<9>(c219);
  const i32 out = (i32)(r2 - (1u << (w - 1))) + cin;
  return {live ? out : 0};
}
FES_DEV fes fes_sq(fes f) { return fes_mul(f, f); }
// f * c for a small constant (|c| < 2^17) and a loose f: one carry round, limbs centred like
// fes_mul's outputs (carries up to 2^18, x 19 into limb 0)
FES_DEV fes fes_mul_small(fes f, i32 c) {
  const int k = fes_lane();
  const bool odd = (k & 1) != 0, live = k < 10;
  const int w = odd ? 25 : 26;
  const i64 h = (i64)(live ? f.v : 0) * (i64)c + ((i64)1 << (w - 1));
  const i32 cy = (i32)(h >> w);
  const i32 r = (i32)((u32)h & ((1u << w) - 1u)) - (1 << (w - 1));
  const i32 cy19 = k == 9 ? cy * 19 : 0;
  const i32 cin = row_shr<1>(cy) | row_shl<9>(cy19);
  return {live ? r + cin : 0};
}
FES_DEV fes fes_add(fes a, fes b) { return {a.v + b.v}; }
FES_DEV fes fes_sub(fes a, fes b) { return {a.v - b.v}; }
FES_DEV fes fes_add_small(fes a, i32 c) { return {fes_lane() == 0 ? a.v + c : a.v}; }   // + c (|c| small)
FES_DEV fes fes_neg(fes a) { return {-a.v}; }

FES_DEV fes fes_sqn(fes f, int n) {
  _Pragma("unroll 1") for (int i = 0; i < n; ++i) f = fes_sq(f);
  return f;
}

// z^(2^252 - 3), the addition chain of fe_pow22523
FES_DEV fes fes_pow22523(fes z) {
  fes z2 = fes_sq(z);
  fes z8 = fes_sqn(z2, 2);
  fes z9 = fes_mul(z, z8);
  fes z11 = fes_mul(z2, z9);
  fes z22 = fes_sq(z11);
  fes t0 = fes_mul(z9, z22);                  // 2^5 - 1
  fes t1 = fes_mul(fes_sqn(t0, 5), t0);       // 2^10 - 1
  fes t2 = fes_mul(fes_sqn(t1, 10), t1);      // 2^20 - 1
  fes t3 = fes_mul(fes_sqn(t2, 20), t2);      // 2^40 - 1
  fes t4 = fes_mul(fes_sqn(t3, 10), t1);      // 2^50 - 1
  fes t5 = fes_mul(fes_sqn(t4, 50), t4);      // 2^100 - 1
  fes t6 = fes_mul(fes_sqn(t5, 100), t5);     // 2^200 - 1
  fes t7 = fes_mul(fes_sqn(t6, 50), t4);      // 2^250 - 1
  return fes_mul(fes_sqn(t7, 2), z);          // 2^252 - 3
}

}  // namespace nwc
