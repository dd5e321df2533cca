// Scalars modulo l = 2^252 + 27742317777372353535851937790883648493 (one per lane).
//
//   sc_lt_l        -- the net A.1 parse rule: ed25519 1.x Signature::from_bytes rejects
//                     sig[63] & 0xE0 (s >= 2^253 > l), dalek check_scalar then requires
//                     s < l; together: accept iff s < l.
//   sc_reduce512   -- Scalar::from_hash: a 512-bit little-endian hash mod l (Barrett,
//                     b = 2^32, k = 8, mu = floor(2^512 / l); HAC Alg. 14.42).
//   sc_recode_*    -- signed fixed-window digits for the uniform (SIMD-friendly) ladder.
#pragma once
#include "consts.h"

namespace nwc {

FE_DEV bool sc_lt_l(const u32 s[8]) {
  // lexicographic compare from the top word
  bool lt = false, eq = true;
  _Pragma("unroll") for (int i = 7; i >= 0; --i) {
    lt = lt || (eq && s[i] < SC_L[i]);
    eq = eq && (s[i] == SC_L[i]);
  }
  return lt;
}

FE_DEV void sc_reduce512(const u32 x[16], u32 r[8]) {
  // q1 = floor(x / b^7): words 7..15 (9 words); q2 = q1 * mu; q3 = floor(q2 / b^9)
  u32 q2[18];
  _Pragma("unroll") for (int i = 0; i < 18; ++i) q2[i] = 0;
  _Pragma("unroll") for (int i = 0; i < 9; ++i) {
    u64 carry = 0;
    _Pragma("unroll") for (int j = 0; j < 9; ++j) {
      u64 t = (u64)x[7 + i] * SC_MU[j] + q2[i + j] + carry;
      q2[i + j] = (u32)t;
      carry = t >> 32;
    }
    q2[i + 9] = (u32)carry;
  }
  // r2 = (q3 * l) mod b^9 ; q3 = q2[9..17]
  u32 r2[9];
  _Pragma("unroll") for (int i = 0; i < 9; ++i) r2[i] = 0;
  _Pragma("unroll") for (int i = 0; i < 9; ++i) {
    u64 carry = 0;
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {
      if (i + j >= 9) break;
      u64 t = (u64)q2[9 + i] * SC_L[j] + r2[i + j] + carry;
      r2[i + j] = (u32)t;
      carry = t >> 32;
    }
    if (i + 8 < 9) r2[i + 8] = (u32)(r2[i + 8] + carry);
  }
  // r = (x mod b^9) - r2 (mod b^9); then at most two subtractions of l
  u32 rr[9];
  u64 borrow = 0;
  _Pragma("unroll") for (int i = 0; i < 9; ++i) {
    u64 t = (u64)x[i] - r2[i] - borrow;
    rr[i] = (u32)t;
    borrow = (t >> 63) & 1;
  }
  _Pragma("unroll") for (int pass = 0; pass < 2; ++pass) {
    // if rr >= l: rr -= l
    u32 tmp[9];
    u64 br = 0;
    _Pragma("unroll") for (int i = 0; i < 9; ++i) {
      u64 t = (u64)rr[i] - (i < 8 ? SC_L[i] : 0u) - br;
      tmp[i] = (u32)t;
      br = (t >> 63) & 1;
    }
    const bool ge = (br == 0);
    _Pragma("unroll") for (int i = 0; i < 9; ++i) rr[i] = ge ? tmp[i] : rr[i];
  }
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r[i] = rr[i];
}

// Signed radix-16 digits of k < 2^253: k = sum d_i 16^i, d_i in [-8, 7], 64 digits.
// Packed as nibbles (d_i + 8) into 8 words, digit i at word i/8, bits 4*(i%8).
FE_DEV void sc_recode_radix16(const u32 k[8], u32 out[8]) {
  i32 carry = 0;
  _Pragma("unroll") for (int w = 0; w < 8; ++w) {
    u32 packed = 0;
    _Pragma("unroll") for (int n = 0; n < 8; ++n) {
      i32 d = (i32)((k[w] >> (4 * n)) & 15u) + carry;
      carry = (d + 8) >> 4;
      d -= carry << 4;
      packed |= (u32)(d + 8) << (4 * n);
    }
    out[w] = packed;
  }
}

// Signed radix-256 digits of s < 2^253: 32 digits in [-128, 127], packed as bytes (d + 128).
FE_DEV void sc_recode_radix256(const u32 s[8], u32 out[8]) {
  i32 carry = 0;
  _Pragma("unroll") for (int w = 0; w < 8; ++w) {
    u32 packed = 0;
    _Pragma("unroll") for (int n = 0; n < 4; ++n) {
      i32 d = (i32)((s[w] >> (8 * n)) & 255u) + carry;
      carry = (d + 128) >> 8;
      d -= carry << 8;
      packed |= (u32)(d + 128) << (8 * n);
    }
    out[w] = packed;
  }
}

// Signed radix-2^16 digits of s < 2^253: 16 digits in [-2^15, 2^15), packed as 16-bit fields
// (d + 2^15), digit 15 in the top half of word 7.
FE_DEV void sc_recode_radix65536(const u32 s[8], u32 out[8]) {
  i32 carry = 0;
  _Pragma("unroll") for (int w = 0; w < 8; ++w) {
    u32 packed = 0;
    _Pragma("unroll") for (int n = 0; n < 2; ++n) {
      i32 d = (i32)((s[w] >> (16 * n)) & 0xFFFFu) + carry;
      carry = (d + 32768) >> 16;
      d -= carry << 16;
      packed |= (u32)(d + 32768) << (16 * n);
    }
    out[w] = packed;
  }
}

// Signed radix-2^BITS digits of s < 2^253 (BITS <= 16): WINDOWS digits in [-2^(BITS-1), 2^(BITS-1)),
// packed as BITS-bit fields (d + 2^(BITS-1)), digit w at bits [BITS w, BITS w + BITS) of out[0..8].
template <int BITS, int WINDOWS>
FE_DEV void sc_recode_radix(const u32 s[8], u32 out[9]) {
  static_assert(BITS * WINDOWS <= 288 && BITS * WINDOWS >= 254, "digit string");
  _Pragma("unroll") for (int i = 0; i < 9; ++i) out[i] = 0;
  i32 carry = 0;
  _Pragma("unroll") for (int w = 0; w < WINDOWS; ++w) {
    const int b = BITS * w, wi = b >> 5, sh = b & 31;
    u32 v = wi < 8 ? s[wi] >> sh : 0u;
    if (sh > 32 - BITS && wi + 1 < 8) v |= s[wi + 1] << (32 - sh);
    i32 d = (i32)(v & ((1u << BITS) - 1u)) + carry;
    carry = (d + (1 << (BITS - 1))) >> BITS;
    d -= carry << BITS;
    const u32 f = (u32)(d + (1 << (BITS - 1)));
    out[wi] |= f << sh;
    if (sh > 32 - BITS) out[wi + 1] |= f >> (32 - sh);
  }
}
// digit w (wave-uniform or per lane) of a radix-2^BITS string
template <int BITS>
FE_DEV i32 digit_at(const u32 d[9], int w) {
  const int b = BITS * w, wi = b >> 5, sh = b & 31;
  u32 lo = d[0], hi = d[1];
  _Pragma("unroll") for (int q = 1; q < 9; ++q) {
    lo = (q == wi) ? d[q] : lo;
    hi = (q + 1 < 9 && q == wi) ? d[q + 1] : hi;
  }
  const u64 v = ((u64)hi << 32 | lo) >> sh;
  return (i32)(v & ((1u << BITS) - 1u)) - (1 << (BITS - 1));
}
FE_DEV void sc_recode_radix4096(const u32 s[8], u32 out[9]) { sc_recode_radix<12, 22>(s, out); }
FE_DEV i32 digit4096_at(const u32 d[9], int w) { return digit_at<12>(d, w); }

// Shift a packed 256-bit digit string left by `bits` (top digits fall out of word 7).
FE_DEV void digits_shl(u32 d[8], int bits) {
  _Pragma("unroll") for (int i = 7; i > 0; --i) d[i] = (d[i] << bits) | (d[i - 1] >> (32 - bits));
  d[0] <<= bits;
}

}  // namespace nwc
