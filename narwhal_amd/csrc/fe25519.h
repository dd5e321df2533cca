// GF(2^255 - 19) arithmetic for gfx950 (MI355X), one field element per lane.
//
// Representation: 10 signed 32-bit limbs, radix 2^25.5 (limb i has weight 2^ceil(25.5 i):
// 26-bit even limbs, 25-bit odd limbs).  Chosen from the int-VALU microbenchmark
// (tools/microbench/int_rates.hip): on gfx950 v_mad_i64_i32 / v_mad_u64_u32
// issue at the same rate as any VOP3 op, so a 100-product schoolbook multiply with 64-bit
// accumulators and NO carry handling inside the product (the sums cannot overflow int64)
// beats a saturated 8x32-bit product-scanning multiply, and fe_add/fe_sub are 10 carry-free
// VOP2 ops instead of a 16-op carry chain.
//
// Bounds (the standard analysis for this radix; exercised by tests/test_gpu_parity.py):
//   "tight"  : |f_i| <= 1.01 * 2^25 (even i) / 1.01 * 2^24 (odd i)     -- fe_mul/fe_sq output
//   "loose"  : |f_i| <= 1.65 * 2^26 / 1.65 * 2^25                      -- allowed mul/sq input
// A sum or difference of up to three tight elements is loose.
//
// The dalek reference semantics these functions implement are restated in SURVEY.md App. A
// (FieldElement::from_bytes ignores bit 255 and accepts y >= p; is_negative = low bit of the
// canonical encoding; sqrt_ratio_i picks the non-negative root).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nwc {

typedef int32_t i32;
typedef int64_t i64;
typedef uint32_t u32;
typedef uint64_t u64;

struct fe { i32 v[10]; };

#define FE_DEV __device__ __forceinline__

FE_DEV fe fe_zero() { fe r; _Pragma("unroll") for (int i = 0; i < 10; ++i) r.v[i] = 0; return r; }
FE_DEV fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }

FE_DEV fe fe_add(const fe& a, const fe& b) {
  fe r; _Pragma("unroll") for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + b.v[i]; return r;
}
FE_DEV fe fe_sub(const fe& a, const fe& b) {
  fe r; _Pragma("unroll") for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] - b.v[i]; return r;
}
FE_DEV fe fe_neg(const fe& a) {
  fe r; _Pragma("unroll") for (int i = 0; i < 10; ++i) r.v[i] = -a.v[i]; return r;
}
// r = c ? b : a  (per-lane select, uniform control flow)
FE_DEV fe fe_select(const fe& a, const fe& b, bool c) {
  fe r; _Pragma("unroll") for (int i = 0; i < 10; ++i) r.v[i] = c ? b.v[i] : a.v[i]; return r;
}

// Column k's accumulator starts at the rounding bias 2^(w_k - 1) (w_k = 26 even, 25 odd), so
// every carry is a floor shift (c = h >> w) and the remainder a mask; the bias is removed once
// at the end, leaving centered limbs in [-2^(w-1), 2^(w-1)] (+ a small incoming carry on limbs
// 1 and 5).  Two interleaved chains (0->1->2->3->4->5, 4->5->6->7->8->9->0) halve the depth.
FE_DEV i64 fe_col_bias(int k) { return (k & 1) ? ((i64)1 << 24) : ((i64)1 << 25); }

FE_DEV fe fe_carry_wide(i64 h[10]) {
  i64 c;
  u32 r[10];
#define FE_FLOOR(i, sh) { c = h[i] >> sh; r[i] = (u32)h[i] & ((1u << sh) - 1u); }
  FE_FLOOR(0, 26); h[1] += c;
  FE_FLOOR(4, 26); h[5] += c;
  FE_FLOOR(1, 25); h[2] += c;
  FE_FLOOR(5, 25); h[6] += c;
  FE_FLOOR(2, 26); h[3] += c;
  FE_FLOOR(6, 26); h[7] += c;
  FE_FLOOR(3, 25); h[4] = (i64)r[4] + c;
  FE_FLOOR(7, 25); h[8] += c;
  FE_FLOOR(4, 26); r[5] += (u32)c;           // c < 2^12 here
  FE_FLOOR(8, 26); h[9] += c;
  FE_FLOOR(9, 25); h[0] = (i64)r[0] + c * 19;
  FE_FLOOR(0, 26); r[1] += (u32)c;           // c < 2^17 here
#undef FE_FLOOR
  fe out;
  _Pragma("unroll") for (int i = 0; i < 10; ++i) out.v[i] = (i32)(r[i] - (u32)fe_col_bias(i));
  return out;
}

}  // namespace nwc
#include "fe_asm.h"
namespace nwc {

// h = f * g.  Column k collects f_i g_j for i + j = k (mod 10); a wrapped term (i + j >= 10)
// carries the factor 19 (2^255 = 19 mod p), and a term with both i, j odd carries 2
// (26 + 25 offsets).  The 19 goes on g (|19 g_j| < 2^31), the 2 on f (|2 f_i| < 2^27).
// The products are one asm block (fe_asm.h, tools/gen_fe_asm.py): per column one
// v_mad_i64_i32 chain seeded with the rounding bias, columns interleaved.
FE_DEV fe fe_mul(const fe& f, const fe& g) {
  i64 h[10];
  fe_mul_wide_asm(f, g, h);
  return fe_carry_wide(h);
}

// h = f^2: 55 distinct products.  Off-diagonal terms carry 2 (symmetry) on the left factor;
// the odd-odd 2 and the wrap 19 go on the right factor (|38 f_j| < 2^31 for odd j).
FE_DEV fe fe_sq(const fe& f) {
  i64 h[10];
  fe_sq_wide_asm(f, h);
  return fe_carry_wide(h);
}

// 2 f^2, doubled before the carry so the result is tight (the 2Z^2 term of point doubling
// is then combined with two more tight terms and stays within the loose bound).  The 2 goes on
// the left factors (|4 f_i| < 2^29).
FE_DEV fe fe_sq2(const fe& f) {
  i64 h[10];
  fe_sq2_wide_asm(f, h);
  return fe_carry_wide(h);
}

FE_DEV fe fe_sqn(fe f, int n) {
  _Pragma("unroll 1") for (int i = 0; i < n; ++i) f = fe_sq(f);
  return f;
}

// Multiply by a small constant (|c| < 2^5): used for d-free formulas only.
FE_DEV fe fe_mul_small(const fe& f, i32 c) {
  i64 h[10];
  _Pragma("unroll") for (int i = 0; i < 10; ++i) h[i] = (i64)f.v[i] * c + fe_col_bias(i);
  return fe_carry_wide(h);
}

// Load the low 255 bits of a little-endian 256-bit value (8 words); bit 255 is ignored and
// values >= p are accepted (reduced implicitly) -- curve25519-dalek FieldElement::from_bytes.
FE_DEV fe fe_from_words(const u32 w[8]) {
  // bit offsets 0,26,51,77,102,128,153,179,204,230; widths 26/25 alternating
  auto bits = [&](int off, int width) -> i32 {
    const int wi = off >> 5, sh = off & 31;
    u64 lo = w[wi];
    u64 hi = (wi + 1 < 8) ? (u64)w[wi + 1] : 0;
    u64 v = (lo | (hi << 32)) >> sh;
    return (i32)(v & ((1ull << width) - 1));
  };
  fe r;
  r.v[0] = bits(0, 26);   r.v[1] = bits(26, 25);  r.v[2] = bits(51, 26);  r.v[3] = bits(77, 25);
  r.v[4] = bits(102, 26); r.v[5] = bits(128, 25); r.v[6] = bits(153, 26); r.v[7] = bits(179, 25);
  r.v[8] = bits(204, 26); r.v[9] = bits(230, 25);
  return r;
}

// Tight form of an element whose limbs are in [0, 2^w) (fe_from_words output): one carry pass
// moving each limb into [-2^(w-1), 2^(w-1)] (+1).  Decoded coordinates are tightened so that every
// coordinate the group formulas see meets the tight bound (2x a tight limb times 19 stays < 2^31).
FE_DEV fe fe_tighten(const fe& f) {
  fe r;
  i32 c = 0;
  _Pragma("unroll") for (int i = 0; i < 10; ++i) {
    const int w = (i & 1) ? 25 : 26;
    const i32 v = f.v[i] + c;
    c = (v + (1 << (w - 1))) >> w;
    r.v[i] = v - (c << w);
  }
  r.v[0] += 19 * c;
  return r;
}

// Canonical encoding (value mod p in [0, p)) as 8 little-endian words.
// Bias by 16p so every limb is non-negative, two carry passes bring every limb into range
// (the second can only ripple out of limb 0), then subtract p once if value >= p.
FE_DEV void fe_to_words(const fe& f, u32 out[8]) {
  i32 h[10];
  h[0] = f.v[0] + ((1 << 30) - 304);
  _Pragma("unroll") for (int i = 1; i < 10; ++i) h[i] = f.v[i] + ((i & 1) ? ((1 << 29) - 16) : ((1 << 30) - 16));
  _Pragma("unroll") for (int pass = 0; pass < 2; ++pass) {
    _Pragma("unroll") for (int i = 0; i < 9; ++i) {
      const int sh = (i & 1) ? 25 : 26;
      i32 c = h[i] >> sh; h[i] -= c << sh; h[i + 1] += c;
    }
    i32 c = h[9] >> 25; h[9] -= c << 25; h[0] += 19 * c;
  }
  // q = floor((v + 19) / 2^255)
  i32 q = (h[0] + 19) >> 26;
  _Pragma("unroll") for (int i = 1; i < 10; ++i) q = (h[i] + q) >> ((i & 1) ? 25 : 26);
  h[0] += 19 * q;
  _Pragma("unroll") for (int i = 0; i < 9; ++i) {
    const int sh = (i & 1) ? 25 : 26;
    i32 c = h[i] >> sh; h[i] -= c << sh; h[i + 1] += c;
  }
  h[9] &= (1 << 25) - 1;
  // pack: limb i occupies bits [off_i, off_i + width_i)
  u32 w[8];
  w[0] = (u32)h[0] | ((u32)h[1] << 26);
  w[1] = ((u32)h[1] >> 6) | ((u32)h[2] << 19);
  w[2] = ((u32)h[2] >> 13) | ((u32)h[3] << 13);
  w[3] = ((u32)h[3] >> 19) | ((u32)h[4] << 6);
  w[4] = (u32)h[5] | ((u32)h[6] << 25);
  w[5] = ((u32)h[6] >> 7) | ((u32)h[7] << 19);
  w[6] = ((u32)h[7] >> 13) | ((u32)h[8] << 12);
  w[7] = ((u32)h[8] >> 20) | ((u32)h[9] << 6);
  _Pragma("unroll") for (int i = 0; i < 8; ++i) out[i] = w[i];
}

FE_DEV bool fe_is_zero(const fe& f) {
  u32 w[8]; fe_to_words(f, w);
  u32 acc = 0; _Pragma("unroll") for (int i = 0; i < 8; ++i) acc |= w[i];
  return acc == 0;
}
FE_DEV bool fe_is_negative(const fe& f) { u32 w[8]; fe_to_words(f, w); return w[0] & 1; }
FE_DEV bool fe_equal(const fe& a, const fe& b) { return fe_is_zero(fe_sub(a, b)); }

// z^(2^252 - 3) = z^((p-5)/8)
FE_DEV fe fe_pow22523(const fe& z) {
  fe z2 = fe_sq(z);
  fe z8 = fe_sqn(z2, 2);
  fe z9 = fe_mul(z, z8);
  fe z11 = fe_mul(z2, z9);
  fe z22 = fe_sq(z11);
  fe t0 = fe_mul(z9, z22);                 // 2^5 - 1
  fe t1 = fe_mul(fe_sqn(t0, 5), t0);       // 2^10 - 1
  fe t2 = fe_mul(fe_sqn(t1, 10), t1);      // 2^20 - 1
  fe t3 = fe_mul(fe_sqn(t2, 20), t2);      // 2^40 - 1
  fe t4 = fe_mul(fe_sqn(t3, 10), t1);      // 2^50 - 1
  fe t5 = fe_mul(fe_sqn(t4, 50), t4);      // 2^100 - 1
  fe t6 = fe_mul(fe_sqn(t5, 100), t5);     // 2^200 - 1
  fe t7 = fe_mul(fe_sqn(t6, 50), t4);      // 2^250 - 1
  return fe_mul(fe_sqn(t7, 2), z);         // 2^252 - 3
}

// z^(p - 2)
FE_DEV fe fe_invert(const fe& z) {
  fe t = fe_sqn(fe_pow22523(z), 3);        // z^(2^255 - 24)
  return fe_mul(t, fe_mul(fe_sq(z), z));   // * z^3
}

}  // namespace nwc
