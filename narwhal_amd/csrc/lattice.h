// Half-size scalars for Ed25519 verification (host + device).
//
// The verification equation e = sB - kA - R = O (dalek verify_strict / the batch leaf,
// SURVEY.md A.3 step 5, A.5) needs 252 shared doublings for the 253-bit k.  Following the
// lattice-reduction idea of Pornin ("Optimized lattice basis reduction in dimension 2, and fast
// Schnorr and EdDSA signature verification", 2020), find (c, d) with
//       d * k = c  (mod 8l),   d odd,   |c|, |d| < 2^146,
// then  [d] e = (d s mod l) B - c A - d R.   Because |E| = 8l and d is odd with 0 < d < l,
// multiplication by d is injective on E (= Z_l x Z_8), so [d] e = O  <=>  e = O: the verdict is
// exactly dalek's, for every A and R including small/mixed-order ones (the modulus is 8l, not l,
// so (dk - c) A = O holds for points with torsion too).  The multi-scalar multiplication then
// needs only 128 doublings (33 radix-16 windows) for typical k.
//
// (c, d) come from the continued-fraction expansion of k / (8l) (Euclid on r_{-1} = 8l,
// r_0 = k with cofactors t): stop at the first r_i < 2^127; if t_i is even, take the best odd
// combination (r_{i-1} - m r_i, t_{i-1} - m t_i).  Quotients are estimated from the top 64 bits
// in double precision and always under-estimated, so each step subtracts q <= floor(r0/r1)
// copies and the remainder sequence is exactly Euclid's.  A lane that does not converge within
// the iteration budget or whose candidate exceeds 2^146 reports failure and is re-verified by the
// full-length ladder.  max(|c|, d) has 127-128 bits typically and its tail falls ~4x per bit
// (tests/test_lattice_host.py): ~0.15 % of k exceed 131 bits, none of 10^6 exceeded 140.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define NWC_HD __host__ __device__ __forceinline__
#else
#define NWC_HD static inline
#endif

namespace nwc {
namespace lat {

typedef uint32_t w32;
typedef uint64_t w64;

constexpr int HALF_BITS = 146;   // accepted |c|, |d| < 2^HALF_BITS (<= 37 radix-16 windows)
constexpr int MAX_ITERS = 192;   // Euclid steps (incl. partial-quotient steps); ~70 on average

// 8l, little-endian words
NWC_HD void eight_l(w32 n[8]) {
  const w32 L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
  w32 carry = 0;
  for (int i = 0; i < 8; ++i) { n[i] = (L[i] << 3) | carry; carry = L[i] >> 29; }
}

NWC_HD bool lt8(const w32 a[8], const w32 b[8]) {
  bool lt = false, eq = true;
  for (int i = 7; i >= 0; --i) { lt = lt || (eq && a[i] < b[i]); eq = eq && (a[i] == b[i]); }
  return lt;
}

// a -= q * b (8 words, a >= q*b guaranteed by the caller)
NWC_HD void submul8(w32 a[8], const w32 b[8], w32 q) {
  w64 borrow = 0;   // amount to subtract from the next word
  for (int i = 0; i < 8; ++i) {
    const w64 p = (w64)q * b[i] + borrow;
    const w32 lo = (w32)p;
    w64 hi = p >> 32;
    const w32 ai = a[i];
    a[i] = ai - lo;
    hi += (ai < lo) ? 1u : 0u;
    borrow = hi;
  }
}

// t -= q * u, 5-word two's complement (wraps mod 2^160; magnitudes stay < 2^159)
NWC_HD void submul5s(w32 t[5], const w32 u[5], w32 q) {
  w64 carry = 0;
  w32 p[5];
  for (int i = 0; i < 5; ++i) { w64 x = (w64)q * u[i] + carry; p[i] = (w32)x; carry = x >> 32; }
  w64 br = 0;
  for (int i = 0; i < 5; ++i) { w64 x = (w64)t[i] - p[i] - br; t[i] = (w32)x; br = (x >> 63) & 1; }
}

NWC_HD bool neg5(const w32 t[5]) { return (t[4] >> 31) != 0; }
NWC_HD void abs5(const w32 t[5], w32 out[5]) {
  const bool n = neg5(t);
  w64 c = 1;
  for (int i = 0; i < 5; ++i) {
    w32 v = n ? ~t[i] : t[i];
    if (n) { w64 x = (w64)v + c; v = (w32)x; c = x >> 32; }
    out[i] = v;
  }
}
NWC_HD int bitlen5(const w32 a[5]) {
  int b = 0;
  for (int i = 0; i < 5; ++i) if (a[i]) b = 32 * i + 32 - __builtin_clz(a[i]);
  return b;
}
NWC_HD int bitlen8(const w32 a[8]) {
  int b = 0;
  for (int i = 0; i < 8; ++i) if (a[i]) b = 32 * i + 32 - __builtin_clz(a[i]);
  return b;
}

// Top 64 bits of a and b at a's top word j (b <= a): floor(a'/(b'+1)) <= floor(a/b), >= 1.
// Branch-free: inside the loop a >= 2^127, so j is one of 3..7 (select chain, no divergence).
NWC_HD double rcp_nr(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(x);
  r = r * (2.0 - x * r);   // Newton: relative error ~ e0^2
  r = r * (2.0 - x * r);
  return r;
#else
  return 1.0 / x;
#endif
}
NWC_HD w32 quot_est(const w32 a[8], const w32 b[8]) {
  w32 ah = a[7], al = a[6], bh = b[7], bl = b[6];
  for (int i = 6; i >= 3; --i) {
    const bool z = ah == 0;
    ah = z ? a[i] : ah;
    al = z ? a[i - 1] : al;
    bh = z ? b[i] : bh;
    bl = z ? b[i - 1] : bl;
  }
  const w64 A = ((w64)ah << 32) | al;
  const w64 B = ((w64)bh << 32) | bl;
  // exact-in-double operands: A truncated to 53 bits, B rounded up to 53 bits (+1); the
  // quotient is scaled by (1 - 2^-40) so reciprocal/rounding error never rounds it up.
  const w64 As = A >> 11, Bs = (B >> 11) + 1;
  double q = (double)As * rcp_nr((double)Bs) * (1.0 - 1.0 / 1099511627776.0);
  w32 qi;
  if (q >= 4294967295.0) qi = 0xFFFFFFFFu;
  else qi = (w32)q;
  return qi < 1 ? 1u : qi;
}

// Result of the reduction.  ok == false -> use the full-length ladder.
struct HalfScalars {
  w32 c[5];      // |c|
  w32 d[5];      // d > 0, odd
  bool c_neg;    // c < 0
  bool ok;
  int bits;      // max(bit length |c|, bit length d)
};

// One step of the exact remainder sequence (a partial-quotient step when q is under-estimated).
NWC_HD void euclid_step(w32 r0[8], w32 r1[8], w32 t0[5], w32 t1[5]) {
  const w32 q = quot_est(r0, r1);
  submul8(r0, r1, q);
  submul5s(t0, t1, q);
  if (lt8(r0, r1)) {
    for (int i = 0; i < 8; ++i) { w32 x = r0[i]; r0[i] = r1[i]; r1[i] = x; }
    for (int i = 0; i < 5; ++i) { w32 x = t0[i]; t0[i] = t1[i]; t1[i] = x; }
  }
}

NWC_HD bool below_2_127(const w32 r[8]) { return (r[7] | r[6] | r[5] | r[4]) == 0 && r[3] < 0x80000000u; }

// 52 bits of x starting at bit s, s in [64, 204] (x < 2^256, so only words 2..7 can be the low one)
NWC_HD w64 bits52(const w32 x[8], int s) {
  const int wi = s >> 5, sh = s & 31;
  w32 a = 0, b = 0, c = 0;
  for (int i = 2; i < 8; ++i) {
    a = i == wi ? x[i] : a;
    b = i == wi + 1 ? x[i] : b;
    c = i == wi + 2 ? x[i] : c;
  }
  const w64 lo = ((w64)b << 32) | a;
  const w64 v = sh ? (lo >> sh) | ((w64)c << (64 - sh)) : lo;
  return v & ((1ull << 52) - 1);
}

// (P - Q) or (Q - P) of P = |a| x, Q = |b| y over N words, mod 2^(32N): one row of the cofactor
// matrix applied to (x, y).  The row's entries have opposite signs (or one is 0), so the
// combination a x + b y is |a| x - |b| y when b <= 0 and |b| y - |a| x otherwise.
template <int N>
NWC_HD void mat_row(const w32 x[N], const w32 y[N], w32 ma, w32 mb, bool b_pos, w32 out[N]) {
  w64 cp = 0, cq = 0;
  w32 p[N], q[N];
  for (int i = 0; i < N; ++i) {
    const w64 u = (w64)ma * x[i] + cp, v = (w64)mb * y[i] + cq;
    p[i] = (w32)u; cp = u >> 32;
    q[i] = (w32)v; cq = v >> 32;
  }
  w64 br = 0;
  for (int i = 0; i < N; ++i) {
    const w32 hi = b_pos ? q[i] : p[i], lo = b_pos ? p[i] : q[i];
    const w64 d = (w64)hi - lo - br;
    out[i] = (w32)d;
    br = (d >> 63) & 1;
  }
}

// Lehmer block (Knuth TAOCP 4.5.2, Algorithm L): run Euclid on the 52-bit leading parts of
// (r0, r1) in double precision (every value an exact integer < 2^53), accept a step only when
// the quotient is certified for the full numbers (Knuth's two-sided test) and the new r1 is
// certainly still >= 2^127 (so the caller's stopping point, the first r1 < 2^127, is never
// skipped), then apply the 2x2 cofactor matrix to (r0, r1) and (t0, t1) once.  The remainder
// sequence stays exactly Euclid's, so (c, d) are bit-identical to reduce<false>.  Returns the
// number of steps taken (0: the caller takes one exact single-precision step).
constexpr int MAX_INNER = 48;    // cofactors < 2^31 bound a block to ~45 steps
constexpr int MAX_OUTER = 96;
NWC_HD int lehmer_block(w32 r0[8], w32 r1[8], w32 t0[5], w32 t1[5]) {
  const int s = bitlen8(r0) - 52;   // r0 > r1 >= 2^127: s >= 76
  double u = (double)bits52(r0, s), v = (double)bits52(r1, s);
  double A = 1, B = 0, C = 0, D = 1;
  // the true new r1 lies above (v' + min(C', D')) 2^s: accept while that is >= 2^127
  const double thr = s >= 127 ? 1.0 : __builtin_ldexp(1.0, 127 - s);
  constexpr double COF_MAX = 2147483648.0;   // 2^31: the matrix entries fit a u32 magnitude
  int steps = 0;
  for (int j = 0; j < MAX_INNER; ++j) {
    const double d1 = v + C, d2 = v + D;
    if (!(d1 > 0 && d2 > 0)) break;
    const double n1 = u + A, n2 = u + B;
    double q = __builtin_floor(n1 * rcp_nr(d1));
    double rem = __builtin_fma(-q, d1, n1);   // exact: a small integer
    if (rem < 0) { q -= 1; rem += d1; }
    if (rem >= d1) q += 1;
    const double rem2 = __builtin_fma(-q, d2, n2);
    if (!(rem2 >= 0 && rem2 < d2)) break;   // quotient not certified
    const double C2 = __builtin_fma(-q, C, A), D2 = __builtin_fma(-q, D, B), v2 = __builtin_fma(-q, v, u);
    if (!(__builtin_fabs(C2) < COF_MAX && __builtin_fabs(D2) < COF_MAX)) break;
    if (!(v2 + __builtin_fmin(C2, D2) >= thr)) break;
    A = C; B = D; C = C2; D = D2; u = v; v = v2;
    ++steps;
  }
  const bool b_pos = B > 0, d_pos = D > 0;
  const w32 ma = (w32)__builtin_fabs(A), mb = (w32)__builtin_fabs(B), mc = (w32)__builtin_fabs(C),
            md = (w32)__builtin_fabs(D);
  w32 n0[8], n1[8], s0[5], s1[5];
  mat_row<8>(r0, r1, ma, mb, b_pos, n0);
  mat_row<8>(r0, r1, mc, md, d_pos, n1);
  mat_row<5>(t0, t1, ma, mb, b_pos, s0);
  mat_row<5>(t0, t1, mc, md, d_pos, s1);
  for (int i = 0; i < 8; ++i) { r0[i] = n0[i]; r1[i] = n1[i]; }
  for (int i = 0; i < 5; ++i) { t0[i] = s0[i]; t1[i] = s1[i]; }
  return steps;
}

template <bool LEHMER = true>
NWC_HD HalfScalars reduce(const w32 k[8]) {
  w32 r0[8], r1[8], t0[5], t1[5];
  eight_l(r0);
  for (int i = 0; i < 8; ++i) r1[i] = k[i];
  for (int i = 0; i < 5; ++i) { t0[i] = 0; t1[i] = 0; }
  t1[0] = 1;
  bool done = false;
  if (LEHMER) {
    for (int it = 0; it < MAX_OUTER; ++it) {
      done = below_2_127(r1);
      if (done) break;
      if (lehmer_block(r0, r1, t0, t1) == 0) euclid_step(r0, r1, t0, t1);
    }
  } else {
    for (int it = 0; it < MAX_ITERS; ++it) {
      done = below_2_127(r1);
      if (done) break;
      euclid_step(r0, r1, t0, t1);
    }
  }
  HalfScalars h;
  h.ok = done;
  // candidate 1: (r1, t1) if t1 odd; else the best odd (r0 - m r1, t0 - m t1)
  w32 c8[8], tc[5];
  if (t1[0] & 1) {
    for (int i = 0; i < 8; ++i) c8[i] = r1[i];
    for (int i = 0; i < 5; ++i) tc[i] = t1[i];
  } else {
    // m ~ (r0 - |t0|) / (r1 + |t1|), estimated in double from the top bits
    w32 a0[5], a1[5];
    abs5(t0, a0);
    abs5(t1, a1);
    auto approx8 = [](const w32 x[8]) -> double {
      double v = 0; for (int i = 7; i >= 0; --i) v = v * 4294967296.0 + (double)x[i]; return v; };
    auto approx5 = [](const w32 x[5]) -> double {
      double v = 0; for (int i = 4; i >= 0; --i) v = v * 4294967296.0 + (double)x[i]; return v; };
    const double num = approx8(r0) - approx5(a0);
    const double den = approx8(r1) + approx5(a1);
    double mf = den > 0 ? num / den : 0.0;
    if (!(mf > 0)) mf = 0;
    if (mf > 4294967294.0) mf = 4294967294.0;
    w32 m = (w32)mf;
    // try m and m + 1, keep the smaller max bit length
    w32 best_c[8], best_t[5];
    int best_bits = 1 << 20;
    for (int dm = 0; dm < 2; ++dm) {
      const w32 mm = m + (w32)dm;
      w32 cc[8], tt[5];
      for (int i = 0; i < 8; ++i) cc[i] = r0[i];
      for (int i = 0; i < 5; ++i) tt[i] = t0[i];
      // cc = r0 - mm r1 (may exceed r0's range only if mm r1 > r0: then skip)
      bool valid = true;
      {
        // compute mm * r1 and compare with r0
        w32 p[9]; w64 carry = 0;
        for (int i = 0; i < 8; ++i) { w64 x = (w64)mm * r1[i] + carry; p[i] = (w32)x; carry = x >> 32; }
        p[8] = (w32)carry;
        if (p[8]) valid = false;
        else {
          bool lt = false, eq = true;
          for (int i = 7; i >= 0; --i) { lt = lt || (eq && r0[i] < p[i]); eq = eq && (r0[i] == p[i]); }
          if (lt) valid = false;
        }
      }
      // |t0 - mm t1| = |t0| + mm |t1| must stay far below 2^159 (no wrap of the 160-bit t)
      if (bitlen5(a1) + (32 - __builtin_clz(mm | 1u)) > 150) valid = false;
      if (!valid) continue;
      submul8(cc, r1, mm);
      submul5s(tt, t1, mm);
      w32 at[5]; abs5(tt, at);
      int bits = bitlen8(cc); const int tb = bitlen5(at); if (tb > bits) bits = tb;
      if (bits < best_bits) {
        best_bits = bits;
        for (int i = 0; i < 8; ++i) best_c[i] = cc[i];
        for (int i = 0; i < 5; ++i) best_t[i] = tt[i];
      }
    }
    if (best_bits == (1 << 20)) { h.ok = false; for (int i = 0; i < 8; ++i) best_c[i] = 0; for (int i = 0; i < 5; ++i) best_t[i] = 1; }
    for (int i = 0; i < 8; ++i) c8[i] = best_c[i];
    for (int i = 0; i < 5; ++i) tc[i] = best_t[i];
  }
  // sign-normalise: d > 0.  c = c8 (>= 0) times sign(t).
  const bool tneg = neg5(tc);
  abs5(tc, h.d);
  h.c_neg = tneg;     // (c, d) -> (-c, -d) when d < 0; c8 >= 0, so then c < 0
  for (int i = 0; i < 5; ++i) h.c[i] = c8[i];
  const int cbits = bitlen5(h.c), dbits = bitlen5(h.d);
  h.bits = cbits > dbits ? cbits : dbits;
  const bool c_small = (c8[5] | c8[6] | c8[7]) == 0 && cbits <= HALF_BITS;
  const bool d_small = dbits <= HALF_BITS;
  if (!(c_small && d_small)) h.ok = false;
  if (c8[0] == 0 && c8[1] == 0 && c8[2] == 0 && c8[3] == 0 && c8[4] == 0) h.c_neg = false;
  return h;
}

}  // namespace lat
}  // namespace nwc
