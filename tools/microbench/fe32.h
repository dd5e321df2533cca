// GF(2^255 - 19) with 8 saturated 32-bit limbs (radix 2^32), the representation SURVEY.md §7
// step 5 names first, measured against the 10 x 25.5-bit one the kernels use (fe25519.h).
//
// Elements are any value < 2^256 (weakly reduced: p <= v < 2^256 is allowed); fe32_canon gives
// [0, p).  Products: 64 v_mad_u64_u32 by product scanning -- column k's products accumulate into
// a 64-bit pair whose carry-out (VCC) is counted in a third word with v_addc_co_u32 (a column of
// up to 8 full 64-bit products needs 67 bits) -- then 2^256 = 38 (mod p): T_lo + 38 T_hi, and the
// carry out of that (<= 39) folded once more.  Experiment only (tools/microbench/fe32.hip); the
// product kernels do not include it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fe32x {

typedef uint32_t u32;
typedef uint64_t u64;

struct fe32 { u32 v[8]; };

#define F32_DEV __device__ __forceinline__

// acc += a * b; hi += carry out of the 64-bit accumulate (VCC)
F32_DEV void mac(u64& acc, u32& hi, u32 a, u32 b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(hi) : "v"(a), "v"(b) : "vcc");
}
// acc += a * b where no carry out is possible
F32_DEV void mac0(u64& acc, u32 a, u32 b) {
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
}

// t = a * b (512 bits), product scanning
F32_DEV void mul512(const fe32& a, const fe32& b, u32 t[16]) {
  u64 acc = 0;
  _Pragma("unroll") for (int k = 0; k < 15; ++k) {
    u32 hi = 0;
    _Pragma("unroll") for (int i = (k < 8 ? 0 : k - 7); i <= (k < 8 ? k : 7); ++i) {
      if (k == 0 || k == 14) mac0(acc, a.v[i], b.v[k - i]);
      else mac(acc, hi, a.v[i], b.v[k - i]);
    }
    t[k] = (u32)acc;
    acc = (acc >> 32) | ((u64)hi << 32);
  }
  t[15] = (u32)acc;
}

// add-with-carry chains (clang's __builtin_addc / __builtin_subc: v_add_co / v_addc_co on VCC)
F32_DEV u32 adc(u32 a, u32 b, u32& c) {
  u32 co;
  const u32 r = __builtin_addc(a, b, c, &co);
  c = co;
  return r;
}
F32_DEV u32 sbb(u32 a, u32 b, u32& c) {
  u32 co;
  const u32 r = __builtin_subc(a, b, c, &co);
  c = co;
  return r;
}

// t = a^2 (512 bits): the 28 cross products by product scanning, the 512-bit sum doubled with
// funnel shifts, then the 8 squares added at words 2i, 2i+1 in one carry chain
F32_DEV void sq512(const fe32& a, u32 t[16]) {
  u64 acc = 0;
  t[0] = 0;
  _Pragma("unroll") for (int k = 1; k < 14; ++k) {
    u32 hi = 0;
    _Pragma("unroll") for (int i = (k < 8 ? 0 : k - 7); i < k - i; ++i) {
      if (k == 1 || k == 13) mac0(acc, a.v[i], a.v[k - i]);
      else mac(acc, hi, a.v[i], a.v[k - i]);
    }
    t[k] = (u32)acc;
    acc = (acc >> 32) | ((u64)hi << 32);
  }
  t[14] = (u32)acc;
  t[15] = (u32)(acc >> 32);
  // double: t <<= 1 (the cross sum is < 2^511)
  _Pragma("unroll") for (int k = 15; k > 0; --k) t[k] = __builtin_amdgcn_alignbit(t[k], t[k - 1], 31);
  t[0] = 0;   // t[0] was 0 before the shift
  u32 c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    const u64 sq = (u64)a.v[i] * a.v[i];
    t[2 * i] = adc(t[2 * i], (u32)sq, c);
    t[2 * i + 1] = adc(t[2 * i + 1], (u32)(sq >> 32), c);
  }
}

// t (512 bits) mod p into < 2^256: T_lo + 38 T_hi (products 38 T_hi_i = h_i 2^32 + l_i added in
// two carry chains), the carry out (< 40) folded once more
F32_DEV fe32 reduce512(const u32 t[16]) {
  u64 p[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) p[i] = (u64)t[8 + i] * 38u;
  fe32 r;
  u32 c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = adc(t[i], (u32)p[i], c);
  u32 top = c;
  c = 0;
  _Pragma("unroll") for (int i = 1; i < 8; ++i) r.v[i] = adc(r.v[i], (u32)(p[i - 1] >> 32), c);
  top += (u32)(p[7] >> 32) + c;   // < 40
  c = 0;
  r.v[0] = adc(r.v[0], top * 38u, c);
  _Pragma("unroll") for (int i = 1; i < 8; ++i) r.v[i] = adc(r.v[i], 0, c);
  r.v[0] += c * 38u;   // a wrap leaves r < 2^11, so this cannot carry
  return r;
}

F32_DEV fe32 fe32_mul(const fe32& a, const fe32& b) {
  u32 t[16];
  mul512(a, b, t);
  return reduce512(t);
}
F32_DEV fe32 fe32_sq(const fe32& a) {
  u32 t[16];
  sq512(a, t);
  return reduce512(t);
}

// fold a carry bit c (weight 2^256) into r: + 38 c, and once more if that wraps
F32_DEV void fold256(fe32& r, u32 c) {
  u32 k = 0;
  r.v[0] = adc(r.v[0], c * 38u, k);
  _Pragma("unroll") for (int i = 1; i < 8; ++i) r.v[i] = adc(r.v[i], 0, k);
  r.v[0] += k * 38u;
}

// a + b (< 2^257) folded into < 2^256
F32_DEV fe32 fe32_add(const fe32& a, const fe32& b) {
  fe32 r;
  u32 c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = adc(a.v[i], b.v[i], c);
  fold256(r, c);
  return r;
}

// a - b: on a borrow the result wrapped by +2^256 = 38 mod p too much; subtract 38 (and once
// more if that borrows), i.e. r = a - b + 2^256 - 38 when a < b, which is = a - b (mod p)
F32_DEV fe32 fe32_sub(const fe32& a, const fe32& b) {
  fe32 r;
  u32 c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) r.v[i] = sbb(a.v[i], b.v[i], c);
  u32 k = 0;
  r.v[0] = sbb(r.v[0], c * 38u, k);
  _Pragma("unroll") for (int i = 1; i < 8; ++i) r.v[i] = sbb(r.v[i], 0, k);
  r.v[0] -= k * 38u;   // a second borrow leaves r >= 2^256 - 38 - ..., so this cannot borrow
  return r;
}

// canonical value in [0, p)
F32_DEV fe32 fe32_canon(const fe32& a) {
  // fold bit 255: v = lo255 + 19 * bit255 < 2^255 + 19
  fe32 r = a;
  const u32 top = r.v[7] >> 31;
  r.v[7] &= 0x7FFFFFFFu;
  u64 c = (u64)top * 19u;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    const u64 s = (u64)r.v[i] + c;
    r.v[i] = (u32)s;
    c = s >> 32;
  }
  // now r < 2^255 + 19: r >= p iff bit 255 of r + 19 is set, and then r - p = (r + 19) - 2^255
  u64 t = 19;
  fe32 w;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    t += r.v[i];
    w.v[i] = (u32)t;
    t >>= 32;
  }
  const bool ge = (w.v[7] >> 31) != 0;
  if (ge) {
    w.v[7] &= 0x7FFFFFFFu;
    r = w;
  }
  return r;
}

}  // namespace fe32x
