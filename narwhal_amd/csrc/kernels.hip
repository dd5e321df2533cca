// HIP kernels of the Narwhal signature-and-digest hot path for gfx950 (MI355X).
//
//   k_build_base_table   i*B, i = 0..128, as affine Niels points (run once at nwc_init)
//   k_verify             one Ed25519 verification equation per lane:
//                          mode STRICT = dalek verify_strict      (crypto/src/lib.rs:200-204)
//                          mode LEAF   = batch leaf, A.5           (crypto/src/lib.rs:206-219)
//                        verdicts leave as a 64-bit ballot per wave (bit i = lane i valid)
//   k_cert_reduce        per-certificate AND of leaf bits + bad-vote bitmap
//   k_cert_index         vote -> certificate index of a host call's votes, from the offsets
//   k_sha512_digest32    Sha512::digest(batch)[..32] per message (worker/src/processor.rs:38)
//   k_keygen_sign        synthetic (pk, sig) generation (RFC 8032 == dalek sign) for workloads
//
// Verification per lane:
//   1. s < l                                       (A.1)
//   2. decompress A and R (dalek quirks)           (A.2)
//   3. STRICT: reject small-order A or R           (A.3 step 3)
//   4. k = SHA-512(R_bytes || A_bytes || M) mod l  (A.3 step 4, raw input bytes)
//   5. R' = k(-A) + sB with a uniform fixed-window ladder: 63 x 4 shared doublings, a signed
//      radix-16 digit of k every 4 bits (9-entry per-lane table of -A multiples) and a signed
//      radix-256 digit of s every 8 bits (129-entry basepoint table in LDS).  Fixed windows keep
//      every lane of a wave on the same add schedule (a w-NAF would make nearly every bit
//      position an add for some lane of 64).
//   6. valid iff R' == R as group elements (X_R' = x_R Z_R', Y_R' = y_R Z_R')  (A.3 step 5)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "fe25519.h"
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"
#include "lattice.h"
#include "fe_sliced.h"
#include "ge_sliced.h"

// Layout and scheduling choices of the half-size ladder were settled by interleaved A/B builds
// (profiles/r02/experiments.md, profiles/r03/experiments.md); the rejected variants live in git
// history and those logs, not as build switches here:
//   - the window's first basepoint DMA is issued before its doublings;
//   - add_lt gathers Z and 2dT only after the extended form is built;
//   - per-lane ladder tables hold 128-B packed entries (one cache line per gather);
//   - R and A are decoded by one noinline call whose points return through scratch.

namespace nwc {

// ------------------------------------------------------------------------------- helpers
__device__ __forceinline__ void load_words8(const uint8_t* p, u32 w[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// Affine Niels form of an extended point (one inversion; setup/generation only).
__device__ ge_niels ge_p3_to_niels(const ge_p3& p) {
  fe zi = fe_invert(p.Z);
  fe x = fe_mul(p.X, zi), y = fe_mul(p.Y, zi);
  ge_niels r;
  r.ypx = fe_add(y, x);
  r.ymx = fe_sub(y, x);
  r.xy2d = fe_mul(fe_mul(x, y), FE_D2);
  return r;
}

__device__ void ge_p3_compress(const ge_p3& p, u32 out[8]) {
  fe zi = fe_invert(p.Z);
  fe x = fe_mul(p.X, zi), y = fe_mul(p.Y, zi);
  fe_to_words(y, out);
  out[7] |= (u32)fe_is_negative(x) << 31;
}

__device__ ge_p3 ge_base_point() {
  ge_p3 b;
  b.X = FE_BASE_X; b.Y = FE_BASE_Y; b.Z = fe_one(); b.T = fe_mul(FE_BASE_X, FE_BASE_Y);
  return b;
}

// SHA-512 of one short message (len <= 111 bytes) given as little-endian words.
__device__ void sha512_one_block(const u32* words, int len, u32 digest_le[16]) {
  uint64_t w[16];
  _Pragma("unroll") for (int i = 0; i < 16; ++i) {
    u32 lo = (2 * i < 28) ? words[2 * i] : 0u;
    u32 hi = (2 * i + 1 < 28) ? words[2 * i + 1] : 0u;
    // mask bytes beyond len, append 0x80
    u32 bl = 0, bh = 0;
    _Pragma("unroll") for (int b = 0; b < 4; ++b) {
      int ilo = 8 * i + b, ihi = 8 * i + 4 + b;
      u32 vlo = (ilo < len) ? ((lo >> (8 * b)) & 0xFF) : (ilo == len ? 0x80u : 0u);
      u32 vhi = (ihi < len) ? ((hi >> (8 * b)) & 0xFF) : (ihi == len ? 0x80u : 0u);
      bl |= vlo << (8 * b);
      bh |= vhi << (8 * b);
    }
    w[i] = be64_from_le32(bl, bh);
  }
  w[15] = (uint64_t)len * 8;
  uint64_t st[8];
  sha512_init_state(st);
  sha512_compress(st, w);
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    digest_le[2 * i] = __builtin_bswap32((u32)(st[i] >> 32));
    digest_le[2 * i + 1] = __builtin_bswap32((u32)st[i]);
  }
}

// ------------------------------------------------------------------------------- base tables
// table[i] = i*B and table[129 + i] = i*(2^132 B), i = 0..128, affine Niels.  One lane per entry.
constexpr int BASE_SPLIT_BITS = 132;
__global__ void k_build_base_table(ge_niels* table) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * 129) return;
  ge_p3 b = ge_base_point();
  if (i >= 129) {
    for (int k = 0; k < BASE_SPLIT_BITS; ++k) b = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(b)));
  }
  const int m = i % 129;
  ge_cached bc = ge_p3_to_cached(b);
  ge_p3 acc = ge_p3_identity();
  for (int bit = 7; bit >= 0; --bit) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((m >> bit) & 1) acc = ge_p1p1_to_p3(ge_add_cached(acc, bc));
  }
  table[i] = ge_p3_to_niels(acc);
}

// Radix-2^24 basepoint tables for the half-size ladder, resident in HBM (2.1 GB of the 288):
// table24[h * B24_ENTRIES + j] = j * (2^(141 h) B), h = 0, 1, j = 0..2^23, affine Niels padded to
// 128 B (8 x dwordx4, the LDS-DMA granule).  e_B = d s mod l (253 bits) splits at 2^141 into
// 6 + 5 signed 24-bit digits: 11 Niels adds per equation for the B term (radix 2^16 took 18).
// Built once per device at init: k_base_pow2 doubles B 141 times on one lane, then one lane
// per entry runs a 23-bit double-and-add (~30 ms for the 16.8M entries).
constexpr int B24_SPLIT_BITS = 141;
constexpr int B24_ENTRIES = (1 << 23) + 1;
struct ge_niels_pad { ge_niels n; u32 pad[2]; };
static_assert(sizeof(ge_niels_pad) == 128, "padded Niels entry");
__global__ void k_base_pow2(ge_p3* out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  ge_p3 b = ge_base_point();
  out[0] = b;
  for (int k = 0; k < B24_SPLIT_BITS; ++k) b = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(b)));
  out[1] = b;
}
__global__ void k_build_base_table24(ge_niels_pad* table, const ge_p3* bases) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * (size_t)B24_ENTRIES) return;
  const int h = i >= (size_t)B24_ENTRIES ? 1 : 0;
  const u32 j = (u32)(i - (size_t)h * B24_ENTRIES);
  const ge_cached bc = ge_p3_to_cached(bases[h]);
  ge_p3 acc = ge_p3_identity();
#pragma unroll 1
  for (int bit = 23; bit >= 0; --bit) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((j >> bit) & 1u) acc = ge_p1p1_to_p3(ge_add_cached(acc, bc));
  }
  table[i].n = ge_p3_to_niels(acc);
  table[i].pad[0] = 0;
  table[i].pad[1] = 0;
}

// ------------------------------------------------------------------------------- committee cache
// nwc_set_committee (config/src/lib.rs:154-156 Committee): per key its decode flags and the
// 129-entry affine Niels table of j * (-A), j = 0..128, resident in L2 (15.5 KB per key).
// Lookup is by exact 32-byte match through an open-addressing hash table built by the host, so
// verdicts never depend on the cache: a cached key has the same decode / small-order flags and
// the same points as decoding it per equation.
struct Committee {
  const u32* keys;          // n x 8 words: the raw 32-byte keys
  const u32* flags;         // n: bit0 = decodes, bit1 = small-order
  const ge_niels* tables;   // n x 129
  const ge_niels_pad* comb;   // n x COMB_PER_KEY (nullptr: committee too large for combs)
  const int32_t* slots;     // hash slot -> key index, -1 = empty
  u32 slot_mask;            // slots - 1 (power of two)
  u32 n;
};
constexpr int COMMITTEE_MAX_PROBE = 16;
__host__ __device__ __forceinline__ u32 committee_hash(const u32 w0, const u32 w1) {
  return (w0 * 0x9E3779B1u) ^ (w1 * 0x85EBCA77u);
}
__device__ __forceinline__ int committee_lookup(const Committee& c, const u32 aw[8]) {
  if (c.n == 0) return -1;
  const u32 h = committee_hash(aw[0], aw[1]);
  int found = -1;
  for (int p = 0; p < COMMITTEE_MAX_PROBE; ++p) {
    const int idx = c.slots[(h + p) & c.slot_mask];
    if (idx < 0) break;
    const u32* k = c.keys + 8 * idx;
    u32 diff = 0;
    _Pragma("unroll") for (int i = 0; i < 8; ++i) diff |= k[i] ^ aw[i];
    if (diff == 0) { found = idx; break; }
  }
  return found;
}

// l * P != O: P has a non-zero 8-torsion component.  dalek's verify_batch scales A_i by
// (z_i k_i mod l), so a key with torsion puts its vote in the randomized domain (SURVEY.md A.4 as
// corrected in round 2; oracle/nwc_oracle.c orc_vote_class).  l = 2^252 + c0 (c0 < 2^125):
// left-to-right double-and-add, 252 doublings and 61 cached additions.  Used once per committee
// key and once per distinct uncached key of a batch-leaf launch, so it is not on the hot path.
__device__ __noinline__ bool ge_has_torsion(const ge_p3& P) {
  const ge_cached pc = ge_p3_to_cached(P);
  ge_p2 acc = ge_p3_to_p2(P);   // bit 252
#pragma unroll 1
  for (int bit = 251; bit >= 0; --bit) {
    ge_p1p1 t = ge_p2_dbl(acc);
    if ((SC_L[bit >> 5] >> (bit & 31)) & 1u) t = ge_add_cached(ge_p1p1_to_p3(t), pc);
    acc = ge_p1p1_to_p2(t);
  }
  return !(fe_is_zero(acc.X) && fe_is_zero(fe_sub(acc.Y, acc.Z)));
}

// Committee key flags: bit0 = decodes, bit1 = small-order, bit2 = has an 8-torsion component.
constexpr u32 KEY_DECODES = 1u, KEY_SMALL_ORDER = 2u, KEY_TORSION = 4u;
// Verdict flags of a cached key for the equation mode: strict rejects small-order A (A.3 step 3),
// the batch leaf rejects torsion-bearing A (randomized domain, answered Err).
__device__ __forceinline__ bool key_flags_ok(u32 fl, bool strict) {
  return (fl & KEY_DECODES) && !(fl & (strict ? KEY_SMALL_ORDER : KEY_TORSION));
}

// One lane per (key, j): table[key][j] = j * (-A_key); lane j == 0 also writes the flags.
__global__ void k_build_key_tables(const u32* __restrict__ keys, u32 n, ge_niels* __restrict__ tables,
                                   u32* __restrict__ flags) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * 129) return;
  const u32 key = t / 129, j = t % 129;
  u32 w[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) w[i] = keys[8 * key + i];
  ge_p3 A[1];
  u32 yc[1][8];
  bool ok[1];
  const u32* const wp[1] = {w};
  ge_decompressN<1>(A, wp, yc, ok);
  const ge_p3 na = ge_p3_neg(A[0]);
  const ge_cached nc = ge_p3_to_cached(na);
  ge_p3 acc = ge_p3_identity();
  for (int bit = 7; bit >= 0; --bit) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((j >> bit) & 1) acc = ge_p1p1_to_p3(ge_add_cached(acc, nc));
  }
  tables[(size_t)key * 129 + j] = ge_p3_to_niels(acc);
  if (j == 0)
    flags[key] = (ok[0] ? KEY_DECODES : 0u) | (ycanon_is_small_order(yc[0]) ? KEY_SMALL_ORDER : 0u) |
                 (ok[0] && ge_has_torsion(A[0]) ? KEY_TORSION : 0u);
}

// ------------------------------------------------------------------------------- committee combs
// Fixed-base combs for the doubling-free committee path (k_verify_comb): for a point P,
//   comb[w * E + j] = j * 2^(BITS w) * P,   w = 0..W-1, j = 0..E-1 = 2^(BITS-1)
// (affine Niels, 128-B entries) so that x * P = sum_w comb[w][d_w] (a negative digit negates the
// entry) for the signed radix-2^BITS digits d_w of any x < 2^253.
//   BaseComb: P = B, radix 2^8, 32 windows (528 KB, nwc_init) -- the latency kernel's basepoint
//   KeyComb:  P = -A_key, radix 2^14, 19 windows (20 MB per key, nwc_set_committee / auto cache)
// One lane per entry: BITS*w doublings of P, a BITS-bit double-and-add, one inversion.
// Radix measured on config 3 with the committee cached (tools/ab_cfg3.sh, profiles/r02/experiments.md):
// key combs 2^12 / 2^14 / 2^16 with a 2^22 basepoint comb: 583-593 / 615 / 528-533 M votes/s.
#ifndef NWC_KEY_COMB_BITS
#define NWC_KEY_COMB_BITS 14
#define NWC_KEY_COMB_WINDOWS 19
#endif
template <int BITS, int WINDOWS>
struct CombShape {
  static constexpr int bits = BITS, windows = WINDOWS, entries = (1 << (BITS - 1)) + 1;
  static constexpr size_t per = (size_t)WINDOWS * entries;
};
using BaseComb = CombShape<8, 32>;
using KeyComb = CombShape<NWC_KEY_COMB_BITS, NWC_KEY_COMB_WINDOWS>;
constexpr size_t COMB_PER_KEY = KeyComb::per;
template <class S>
__global__ void k_build_comb(const u32* __restrict__ keys, u32 n, ge_niels_pad* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)(keys ? n : 1u) * S::per) return;
  const u32 key = (u32)(t / S::per), r = (u32)(t % S::per);
  const int w = (int)(r / S::entries), j = (int)(r % S::entries);
  ge_p3 P;
  if (keys) {
    u32 kw[8];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) kw[i] = keys[8 * key + i];
    u32 yc[1][8];
    bool ok[1];
    const u32* const wp[1] = {kw};
    ge_decompressN<1>(&P, wp, yc, ok);
    P = ge_p3_neg(P);
  } else {
    P = ge_base_point();
  }
  for (int k = 0; k < S::bits * w; ++k) P = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(P)));
  const ge_cached pc = ge_p3_to_cached(P);
  ge_p3 acc = ge_p3_identity();
  for (int bit = S::bits - 1; bit >= 0; --bit) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((j >> bit) & 1) acc = ge_p1p1_to_p3(ge_add_cached(acc, pc));
  }
  out[t].n = ge_p3_to_niels(acc);
  out[t].pad[0] = 0;
  out[t].pad[1] = 0;
}

// Key combs in two passes (the same points as k_build_comb<S>, ~4x less work): one lane per key
// decodes it and doubles -A into the window bases 2^(BITS w) (-A); then one lane per entry runs a
// BITS-bit double-and-add from its window's base and one inversion.
template <class S>
__global__ void k_comb_key_bases(const u32* __restrict__ keys, u32 n, ge_p3* __restrict__ bases) {
  const u32 key = blockIdx.x * blockDim.x + threadIdx.x;
  if (key >= n) return;
  u32 kw[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) kw[i] = keys[8 * key + i];
  u32 yc[1][8];
  bool ok[1];
  const u32* const wp[1] = {kw};
  ge_p3 P;
  ge_decompressN<1>(&P, wp, yc, ok);
  P = ge_p3_neg(P);
#pragma unroll 1
  for (int w = 0; w < S::windows; ++w) {
    bases[(size_t)key * S::windows + w] = P;
#pragma unroll 1
    for (int k = 0; k < S::bits; ++k) P = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(P)));
  }
}
// Entries of a comb window built in runs of COMB_RUN consecutive multiples per lane, with one
// inversion per run (Montgomery's trick): entry j0 = j0 * base by double-and-add, then each next
// entry is the previous + base; the projective (X, Y, Z) of every entry is parked in its own output
// slot (120 of its 128 bytes) while the running product of the Z goes forward, one inversion, and
// the backward pass turns each slot into its affine Niels form.  Per entry ~1/8 of a scalar
// multiplication and of an inversion plus one addition and ~5 products, instead of a 14-bit
// double-and-add and an inversion each (round 3's one-lane-per-entry builder): nwc_set_committee,
// the auto key cache and the launch keys build their 20-MB combs this way.
constexpr int COMB_RUN = 8;
struct CombRunPark { fe X, Y, Z; u32 pad[2]; };
static_assert(sizeof(CombRunPark) == sizeof(ge_niels_pad), "parked entry fits its slot");
template <class S>
__device__ __forceinline__ void comb_build_run(const ge_p3* __restrict__ bases, ge_niels_pad* __restrict__ out, size_t run) {
  constexpr u32 RUNS_PER_WINDOW = (S::entries + COMB_RUN - 1) / COMB_RUN;
  const size_t kw = run / RUNS_PER_WINDOW;   // key * windows + w
  const u32 j0 = (u32)(run % RUNS_PER_WINDOW) * COMB_RUN;
  const ge_p3 base = bases[kw];
  const ge_cached pc = ge_p3_to_cached(base);
  ge_p3 acc = ge_p3_identity();
#pragma unroll 1
  for (int bit = S::bits - 1; bit >= 0; --bit) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((j0 >> bit) & 1) acc = ge_p1p1_to_p3(ge_add_cached(acc, pc));
  }
  ge_niels_pad* const dst = out + kw * S::entries + j0;
  CombRunPark* const park = reinterpret_cast<CombRunPark*>(dst);
  const int cnt = (int)min<u32>(COMB_RUN, S::entries - j0);
  fe prod[COMB_RUN];
  _Pragma("unroll") for (int k = 0; k < COMB_RUN; ++k) {
    if (k < cnt) {
      park[k].X = acc.X;
      park[k].Y = acc.Y;
      park[k].Z = acc.Z;
      prod[k] = k ? fe_mul(prod[k - 1], acc.Z) : acc.Z;
      if (k + 1 < cnt) acc = ge_p1p1_to_p3(ge_add_cached(acc, pc));
    }
  }
  fe inv = fe_invert(prod[cnt - 1]);
  _Pragma("unroll") for (int k = COMB_RUN - 1; k >= 0; --k) {
    if (k < cnt) {
      const fe X = park[k].X, Y = park[k].Y, Z = park[k].Z;
      const fe zi = k ? fe_mul(inv, prod[k - 1]) : inv;
      if (k) inv = fe_mul(inv, Z);
      const fe x = fe_mul(X, zi), y = fe_mul(Y, zi);
      ge_niels_pad e;
      e.n.ypx = fe_add(y, x);
      e.n.ymx = fe_sub(y, x);
      e.n.xy2d = fe_mul(fe_mul(x, y), FE_D2);
      e.pad[0] = 0;
      e.pad[1] = 0;
      dst[k] = e;
    }
  }
}
// Combs of keys [k0, k1) from their window bases (bases and out indexed from key 0); k0/k1 come
// from the host, or from range[1] / range[0] on the device when range is not null (launch keys).
template <class S>
__global__ void k_build_comb_from_bases(const ge_p3* __restrict__ bases, u32 k0, u32 k1, const u32* range,
                                        ge_niels_pad* __restrict__ out) {
  constexpr u32 RUNS_PER_WINDOW = (S::entries + COMB_RUN - 1) / COMB_RUN;
  if (range) {
    k0 = range[1];
    k1 = range[0];
  }
  const size_t lo = (size_t)k0 * S::windows * RUNS_PER_WINDOW, hi = (size_t)k1 * S::windows * RUNS_PER_WINDOW;
  for (size_t r = lo + (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < hi; r += (size_t)gridDim.x * blockDim.x)
    comb_build_run<S>(bases, out, r);
}

// Basepoint comb for the throughput committee kernel: comb16[w * E + j] = j * 2^(BITS w) * B,
// w < WINDOWS, j = 0..2^(BITS-1) (E entries per window; radix 2^22: 12 x 2,097,153 entries =
// 3.2 GB of the 288 GB HBM): s*B is 12 additions instead of 16 at radix 2^16 (67 MB; 541 -> 590 M
// votes/s on config 3, profiles/r02/experiments.md; 2^24 / 11 windows / 11.8 GB gained nothing
// more).  Built once at nwc_init (~60 ms): k_bcomb_bases doubles B into the window bases on one
// lane, then one lane per entry runs a BITS-bit double-and-add and one inversion.
#ifndef NWC_BCOMB_BITS
#define NWC_BCOMB_BITS 22
#endif
#ifndef NWC_BCOMB_WINDOWS
#define NWC_BCOMB_WINDOWS 12
#endif
using BCombShape = CombShape<NWC_BCOMB_BITS, NWC_BCOMB_WINDOWS>;
constexpr int COMB16_WINDOWS = BCombShape::windows, COMB16_ENTRIES = BCombShape::entries;
constexpr size_t COMB16_TOTAL = BCombShape::per;
__global__ void k_bcomb_bases(ge_p3* out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  ge_p3 b = ge_base_point();
  for (int w = 0; w < COMB16_WINDOWS; ++w) {
    out[w] = b;
    for (int k = 0; k < NWC_BCOMB_BITS; ++k) b = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(b)));
  }
}
__global__ void k_build_comb16(ge_niels_pad* __restrict__ out, const ge_p3* __restrict__ bases) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= COMB16_TOTAL) return;
  const int w = (int)(t / COMB16_ENTRIES), j = (int)(t % COMB16_ENTRIES);
  const ge_cached pc = ge_p3_to_cached(bases[w]);
  ge_p3 acc = ge_p3_identity();
#pragma unroll 1
  for (int bit = NWC_BCOMB_BITS - 1; bit >= 0; --bit) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((j >> bit) & 1) acc = ge_p1p1_to_p3(ge_add_cached(acc, pc));
  }
  out[t].n = ge_p3_to_niels(acc);
  out[t].pad[0] = 0;
  out[t].pad[1] = 0;
}

// ------------------------------------------------------------------------------- ladder
// Per-lane table of the variable base in global scratch, lane-contiguous: 9 entries x 128 B
// (a cached point packed into 8 x dwordx4).  A lookup reads one lane's 128 contiguous bytes,
// so a wave touches ~64 lines per lookup instead of the whole wave's table (the compiler's
// private memory interleaves lanes dword by dword).
constexpr int TAB_ENTRIES = 9;
// Packed entries: each coordinate's ten limbs, made non-negative, in 32 bytes (fields of 26, 26,
// 26, 25, 26, 25, 26, 25, 26, 25 bits at bit offsets 0, 26, 52, 78, 103, 129, 154, 180, 205, 231;
// limb 1 keeps one slack bit for the final carry).  An entry is 128 B on a 128-B boundary, so a
// gather of one entry touches exactly one cache line (160-B entries touch two).
constexpr int TAB_U4_PER_ENTRY = 8;

// f (limbs |f_i| < 2^26.5 even / 2^25.5 odd: sums of two tight elements) + 2p, floor-carried to
// limbs in [0, 2^26) / [0, 2^25) (limb 1 < 2^25 + 2), packed into two uint4.
__device__ __forceinline__ void fe_pack(const fe& f, uint4& lo, uint4& hi) {
  u32 h[10];
  i32 c = 0;
  _Pragma("unroll") for (int i = 0; i < 10; ++i) {
    const int w = (i & 1) ? 25 : 26;
    const i32 bias = i == 0 ? 2 * ((1 << 26) - 19) : 2 * ((1 << w) - 1);
    const i32 v = f.v[i] + bias + c;   // > 0
    c = v >> w;
    h[i] = (u32)v & ((1u << w) - 1u);
  }
  h[0] += 19u * (u32)c;                // c <= 3: h[0] < 2^26 + 57
  h[1] += h[0] >> 26;
  h[0] &= (1u << 26) - 1u;
  lo.x = h[0] | (h[1] << 26);
  lo.y = (h[1] >> 6) | (h[2] << 20);
  lo.z = (h[2] >> 12) | (h[3] << 14);
  lo.w = (h[3] >> 18) | (h[4] << 7);
  hi.x = (h[4] >> 25) | (h[5] << 1) | (h[6] << 26);
  hi.y = (h[6] >> 6) | (h[7] << 20);
  hi.z = (h[7] >> 12) | (h[8] << 13);
  hi.w = (h[8] >> 19) | (h[9] << 7);
}
// Unpacked limbs are in [0, 2^26) / [0, 2^25 + 2): within the multiplier's loose input bound
// (including the 19x on the right operand).
__device__ __forceinline__ fe fe_unpack(const uint4& lo, const uint4& hi) {
  constexpr u32 M26 = (1u << 26) - 1u, M25 = (1u << 25) - 1u;
  fe r;
  r.v[0] = (i32)(lo.x & M26);
  r.v[1] = (i32)(__builtin_amdgcn_alignbit(lo.y, lo.x, 26) & M26);
  r.v[2] = (i32)(__builtin_amdgcn_alignbit(lo.z, lo.y, 20) & M26);
  r.v[3] = (i32)(__builtin_amdgcn_alignbit(lo.w, lo.z, 14) & M25);
  r.v[4] = (i32)(__builtin_amdgcn_alignbit(hi.x, lo.w, 7) & M26);
  r.v[5] = (i32)((hi.x >> 1) & M25);
  r.v[6] = (i32)(__builtin_amdgcn_alignbit(hi.y, hi.x, 26) & M26);
  r.v[7] = (i32)(__builtin_amdgcn_alignbit(hi.z, hi.y, 20) & M25);
  r.v[8] = (i32)(__builtin_amdgcn_alignbit(hi.w, hi.z, 13) & M26);
  r.v[9] = (i32)(hi.w >> 7);
  return r;
}
constexpr size_t TAB_BYTES_PER_LANE = TAB_ENTRIES * TAB_U4_PER_ENTRY * 16;   // 1440 (1152 packed)

struct LaneTable {
  uint4* p;
  __device__ __forceinline__ void store(int e, const ge_cached& c) const {
    const fe* co = &c.YpX;
    _Pragma("unroll") for (int k = 0; k < 4; ++k) {
      uint4 lo, hi;
      fe_pack(co[k], lo, hi);
      p[e * 8 + 2 * k] = lo;
      p[e * 8 + 2 * k + 1] = hi;
    }
  }
  __device__ __forceinline__ ge_cached load(int e) const {
    ge_cached c;
    fe* co = &c.YpX;
    _Pragma("unroll") for (int k = 0; k < 4; ++k) co[k] = fe_unpack(p[e * 8 + 2 * k], p[e * 8 + 2 * k + 1]);
    return c;
  }
};

// Coordinate k (0 YpX, 1 YmX, 2 Z, 3 T2d) of entry e: 40 bytes at an 8-byte-aligned offset
// (packed: 32 bytes at a 32-byte-aligned offset).
__device__ __forceinline__ fe lt_load_fe(const LaneTable& tab, int e, int k) {
  return fe_unpack(tab.p[e * 8 + 2 * k], tab.p[e * 8 + 2 * k + 1]);
}
// The ladder's first entry as a completed point: the table's coordinates re-centred first when
// packed (2Z of limbs up to 2^27 would exceed the multiplier's right-operand bound).
__device__ __forceinline__ ge_cached lt_first(const LaneTable& tab, int e) {
  ge_cached c = tab.load(e);
  c.YpX = fe_tighten(c.YpX);
  c.YmX = fe_tighten(c.YmX);
  c.Z = fe_tighten(c.Z);
  c.T2d = fe_tighten(c.T2d);
  return c;
}

// t + (neg ? -q : q) for q = tab[e], t completed (p1p1), result completed: 8M, with the entry
// read coordinate by coordinate and the extended form built pairwise, so at most ~2 points'
// worth of field elements are live (the 3-waves-per-SIMD register budget).  -q swaps Y+X / Y-X
// (a per-lane address choice) and negates 2dT (the sign flips on the sum/difference of zz2, tt).
__device__ __forceinline__ ge_p1p1 add_lt(const ge_p1p1& t, const LaneTable& tab, int e, bool neg) {
  const fe qa = lt_load_fe(tab, e, neg ? 1 : 0);
  const fe qb = lt_load_fe(tab, e, neg ? 0 : 1);
  const fe X3 = fe_mul(t.X, t.T), Y3 = fe_mul(t.Z, t.Y);
  const fe a = fe_add(Y3, X3), b = fe_sub(Y3, X3);
  const fe Z3 = fe_mul(t.Z, t.T), T3 = fe_mul(t.X, t.Y);
  __builtin_amdgcn_sched_barrier(0);
  const fe qz = lt_load_fe(tab, e, 2);
  const fe qt = lt_load_fe(tab, e, 3);
  const fe pp = fe_mul(a, qa), mm = fe_mul(b, qb);
  ge_p1p1 r;
  r.X = fe_sub(pp, mm);
  r.Y = fe_add(pp, mm);
  const fe zz = fe_mul(Z3, qz);
  const fe zz2 = fe_add(zz, zz);
  fe tt = fe_mul(T3, qt);
  tt = fe_select(tt, fe_neg(tt), neg);
  r.Z = fe_add(zz2, tt);
  r.T = fe_sub(zz2, tt);
  return r;
}

// The entry's first two coordinates (Y+X, Y-X, swapped when neg), packed: 4 x uint4.
__device__ __forceinline__ void lt_load_ab(const LaneTable& tab, int e, bool neg, uint4 ab[4]) {
  const int ka = neg ? 1 : 0, kb = neg ? 0 : 1;
  ab[0] = tab.p[e * 8 + 2 * ka];
  ab[1] = tab.p[e * 8 + 2 * ka + 1];
  ab[2] = tab.p[e * 8 + 2 * kb];
  ab[3] = tab.p[e * 8 + 2 * kb + 1];
}
// The whole packed entry (Y+X, Y-X swapped when neg, Z, 2dT: 8 x uint4) gathered ahead of its
// add, so that the add issues no load of its own: with a partial prefetch the add's own Z / 2dT
// loads were the newest in flight, and the in-order vmcnt wait for them also waited for the next
// entry's prefetch (k_verify_straus: consecutive additions with no doubling between them).
__device__ __forceinline__ void lt_load_full(const LaneTable& tab, int e, bool neg, uint4 q[8]) {
  lt_load_ab(tab, e, neg, q);
  q[4] = tab.p[e * 8 + 4];
  q[5] = tab.p[e * 8 + 5];
  q[6] = tab.p[e * 8 + 6];
  q[7] = tab.p[e * 8 + 7];
}
__device__ __forceinline__ ge_p1p1 add_lt_full(const ge_p1p1& t, const uint4 q[8], bool neg) {
  const fe X3 = fe_mul(t.X, t.T), Y3 = fe_mul(t.Z, t.Y);
  const fe a = fe_add(Y3, X3), b = fe_sub(Y3, X3);
  const fe Z3 = fe_mul(t.Z, t.T), T3 = fe_mul(t.X, t.Y);
  const fe pp = fe_mul(a, fe_unpack(q[0], q[1])), mm = fe_mul(b, fe_unpack(q[2], q[3]));
  ge_p1p1 r;
  r.X = fe_sub(pp, mm);
  r.Y = fe_add(pp, mm);
  const fe zz = fe_mul(Z3, fe_unpack(q[4], q[5]));
  const fe zz2 = fe_add(zz, zz);
  fe tt = fe_mul(T3, fe_unpack(q[6], q[7]));
  tt = fe_select(tt, fe_neg(tt), neg);
  r.Z = fe_add(zz2, tt);
  r.T = fe_sub(zz2, tt);
  return r;
}

// tab[j] = j * P for j = 0..8 (tab[0] = identity)
__device__ __forceinline__ void build_table(const LaneTable& tab, const ge_p3& P) {
  ge_cached p1 = ge_p3_to_cached(P);
  tab.store(0, ge_cached_identity());
  tab.store(1, p1);
  ge_p3 pj = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(P)));
  tab.store(2, ge_p3_to_cached(pj));
#pragma unroll 1
  for (int j = 3; j < TAB_ENTRIES; ++j) {
    pj = ge_p1p1_to_p3(ge_add_cached(pj, p1));
    tab.store(j, ge_p3_to_cached(pj));
  }
}

__device__ __forceinline__ void ladder_double4(ge_p1p1& t, ge_p3& acc) {
  ge_p2 p2 = ge_p1p1_to_p2(t);
  t = ge_p2_dbl(p2);
  p2 = ge_p1p1_to_p2(t);
  t = ge_p2_dbl(p2);
  p2 = ge_p1p1_to_p2(t);
  t = ge_p2_dbl(p2);
  p2 = ge_p1p1_to_p2(t);
  t = ge_p2_dbl(p2);
  acc = ge_p1p1_to_p3(t);
}

// ---- full-length ladder: R' = k*P + s*B, 64 radix-16 windows (the fallback path) -------------
__device__ __forceinline__ ge_p2 double_scalarmult(const LaneTable& tab, u32 kd[8], u32 sd[8],
                                                   const ge_niels* sB) {
  ge_p3 acc = ge_p3_identity();
  ge_p1p1 t;
  i32 dk = (i32)(kd[7] >> 28) - 8;
  digits_shl(kd, 4);
  ge_cached nxt = tab.load(dk < 0 ? -dk : dk);
#pragma unroll 1
  for (int w = 63; w >= 0; --w) {
    const ge_cached cur = ge_cached_cneg(nxt, dk < 0);
    if (w > 0) {
      dk = (i32)(kd[7] >> 28) - 8;
      digits_shl(kd, 4);
      nxt = tab.load(dk < 0 ? -dk : dk);
    }
    if (w != 63) ladder_double4(t, acc);
    t = ge_add_cached(acc, cur);
    if ((w & 1) == 0) {
      const i32 ds = (i32)(sd[7] >> 24) - 128;
      digits_shl(sd, 8);
      const ge_niels nb = sB[ds < 0 ? -ds : ds];
      acc = ge_p1p1_to_p3(t);
      t = ge_add_niels(acc, ge_niels_cneg(nb, ds < 0));
    }
  }
  return ge_p1p1_to_p2(t);
}

// ---- half-size ladder: Q = eB*B + c'*PA + d*PR over W radix-16 windows -----------------------
// W is wave-uniform: the smallest W in [33, 37] with |c|, d < 2^(4W-1) for every lane of the
// wave (max(|c|, d) has 127-128 bits typically; ~9 % of waves hold a lane of 132+ bits and run
// 34-35 windows, and only |c| or d >= 2^147 -- never seen in 10^6 samples -- leaves the
// half-size path).  The basepoint scalar eB = d s mod l is split at 2^132 into two 9-digit
// radix-2^16 strings added at the windows w = 32, 28, ..., 0 from tables in HBM.
// Digit streams are packed so the next digit is always in the top nibble/byte of word 4 and is
// consumed by shifting the 160-bit string left:
//   Digits16  {w[5], top}: signed radix-16 digits of x < 2^(4W-1): digits 0..W-2 in [-8, 7] as
//     nibbles d+8 (digit W-2 in the top nibble), digit W-1 = top in [0, 8].
//   Digits256 {w[5]}: signed radix-256 digits as bytes d+128, the first digit to use in the top byte.
// The accumulator between operations is kept in completed (p1p1) form `t`: an add converts it to
// extended (4M) because the addition needs T; a doubling only needs (X:Y:Z) (3M).  So the last
// add of each window feeds the next window's doublings at 3M instead of 4M.
constexpr int HALF_WINDOWS_MIN = 33, HALF_WINDOWS_MAX = 37;
struct Digits16 { u32 w[5]; i32 top; };
struct Digits256 { u32 w[5]; };

__device__ __forceinline__ i32 next16(Digits16& x) {
  const i32 d = (i32)(x.w[4] >> 28) - 8;
  _Pragma("unroll") for (int i = 4; i > 0; --i) x.w[i] = (x.w[i] << 4) | (x.w[i - 1] >> 28);
  x.w[0] <<= 4;
  return d;
}
__device__ __forceinline__ i32 next256(Digits256& x) {
  const i32 d = (i32)(x.w[4] >> 24) - 128;
  _Pragma("unroll") for (int i = 4; i > 0; --i) x.w[i] = (x.w[i] << 8) | (x.w[i - 1] >> 24);
  x.w[0] <<= 8;
  return d;
}
// 160-bit left shift by a wave-uniform bit count s in [0, 32]
__device__ __forceinline__ void shl160_dyn(u32 w[5], u32 s) {
  if (s == 32) {
    _Pragma("unroll") for (int i = 4; i > 0; --i) w[i] = w[i - 1];
    w[0] = 0;
  } else if (s) {
    _Pragma("unroll") for (int i = 4; i > 0; --i) w[i] = (w[i] << s) | (w[i - 1] >> (32 - s));
    w[0] <<= s;
  }
}

// Signed radix-16 digits of x < 2^(4W-1) for a wave-uniform W in [33, 37].
__device__ __forceinline__ Digits16 recode16(const u32 x[5], int W) {
  Digits16 r;
  _Pragma("unroll") for (int i = 0; i < 5; ++i) r.w[i] = 0;
  r.top = 0;
  i32 carry = 0;
  _Pragma("unroll") for (int i = 0; i < HALF_WINDOWS_MAX - 1; ++i) {
    const i32 v = (i32)((x[i >> 3] >> (4 * (i & 7))) & 15u) + carry;
    if (i == W - 1) r.top = v;
    carry = (v + 8) >> 4;
    const i32 d = v - (carry << 4);
    const int pos = i + 4;   // digit 35 in the top nibble of word 4
    r.w[pos >> 3] |= (u32)(d + 8) << (4 * (pos & 7));
  }
  if (W == HALF_WINDOWS_MAX) r.top = (i32)((x[4] >> 16) & 15u) + carry;
  // move digit W-2 to the top nibble (digits >= W-1 leave the string)
  shl160_dyn(r.w, 4u * (u32)(HALF_WINDOWS_MAX - W));
  return r;
}
// Signed radix-256 digits of x < 2^(8 ndig - 1) (ndig <= 19, d in [-128, 128]) as bytes d+128
// with digit ndig-1 in the top byte of word 4.  ndig may be wave-uniform dynamic.
__device__ __forceinline__ Digits256 recode256(const u32 x[5], int ndig) {
  Digits256 r;
  _Pragma("unroll") for (int i = 0; i < 5; ++i) r.w[i] = 0;
  i32 carry = 0;
  _Pragma("unroll") for (int i = 0; i < 19; ++i) {
    i32 d = (i32)((x[i >> 2] >> (8 * (i & 3))) & 255u) + carry;
    carry = (d + 128) >> 8;
    d -= carry << 8;
    const int pos = i + 1;   // digit 18 in the top byte of word 4
    r.w[pos >> 2] |= (u32)(d + 128) << (8 * (pos & 3));
  }
  shl160_dyn(r.w, 8u * (u32)(19 - ndig));
  return r;
}

// Signed radix-2^24 digits of the two halves of e_B (tables in HBM): lo < 2^141 has 6 digits
// (windows 30, 24, ..., 0), hi < 2^112 has 5 (windows 24, ..., 0); digits in [-2^23, 2^23) except
// the top one of each half, which takes the final carry (<= 2^21 + 1 and 2^16 + 1).  A queue of
// registers, next digit last: consuming one is five moves, no dynamic register indexing.
constexpr int B24_LO_DIGITS = 6, B24_HI_DIGITS = 5;
struct Digits24 { i32 d[B24_LO_DIGITS]; };
template <int N>
__device__ __forceinline__ Digits24 recode24(const u32 x[5]) {
  static_assert(N >= 1 && N <= B24_LO_DIGITS, "digit count");
  constexpr int OFF = B24_LO_DIGITS - N;   // digit i sits at queue slot i + OFF (top digit last)
  Digits24 r;
  _Pragma("unroll") for (int i = 0; i < OFF; ++i) r.d[i] = 0;
  i32 carry = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) {
    const int bit = 24 * i, wi = bit >> 5, sh = bit & 31;
    u32 v = x[wi] >> sh;
    if (sh > 8 && wi + 1 < 5) v |= x[wi + 1] << (32 - sh);
    const i32 t = (i32)(v & 0xFFFFFFu) + carry;
    if (i == N - 1) {
      r.d[i + OFF] = t;
    } else {
      carry = (t + (1 << 23)) >> 24;
      r.d[i + OFF] = t - (carry << 24);
    }
  }
  return r;
}
// Digit strings parked in LDS for the ladder (k_verify's 256-thread blocks), so no VGPR holds them
// across the windows: per thread, word k at p[k * 256] (a wave's access is one conflict-free 256 B
// row).  Words [0, 6): e_B's low-half radix-2^24 digits, [6, 11): its high half, [11, 16) and
// [16, 21): the Digits16 strings of |c| and d (the uncached ladder).
constexpr int BD_HI = B24_LO_DIGITS, BD_C = BD_HI + B24_HI_DIGITS, BD_D = BD_C + 5;
constexpr int BASE_DIGIT_WORDS = BD_D + 5;   // 21 words per thread
struct BaseDigits { i32* p; };
__device__ __forceinline__ void park16(BaseDigits bd, int off, const Digits16& x) {
  _Pragma("unroll") for (int i = 0; i < 5; ++i) bd.p[(off + i) * 256] = (i32)x.w[i];
}
// digit of window w (w <= W - 2) of a parked Digits16 string: nibble w + 41 - W (recode16's layout)
__device__ __forceinline__ i32 digit16(BaseDigits bd, int off, int w, int W) {
  const int pos = w + 41 - W;
  return (i32)(((u32)bd.p[(off + (pos >> 3)) * 256] >> (4 * (pos & 7))) & 15u) - 8;
}
__device__ __forceinline__ void base_digits_park(BaseDigits bd, const Digits24& el, const Digits24& eh) {
  _Pragma("unroll") for (int i = 0; i < B24_LO_DIGITS; ++i) bd.p[i * 256] = el.d[i];
  _Pragma("unroll") for (int i = 0; i < B24_HI_DIGITS; ++i) bd.p[(BD_HI + i) * 256] = eh.d[i + B24_LO_DIGITS - B24_HI_DIGITS];
}
__device__ __forceinline__ i32 next24(Digits24& x) {
  const i32 d = x.d[B24_LO_DIGITS - 1];
  _Pragma("unroll") for (int i = B24_LO_DIGITS - 1; i > 0; --i) x.d[i] = x.d[i - 1];
  x.d[0] = 0;
  return d;
}
// window w of the half-size ladder consumes 2 (w = 0, 6, .., 24), 1 (w = 30) or 0 basepoint digits
__device__ __forceinline__ int base_window_digits(int w) {
  return (w % 6 != 0 || w > 6 * (B24_LO_DIGITS - 1)) ? 0 : (w > 6 * (B24_HI_DIGITS - 1) ? 1 : 2);
}

// LDS staging of basepoint-table entries fetched by LDS-DMA (global_load_lds_dwordx4): each wave
// owns 16 x 64 uint4; chunk c of entry e of lane l sits at stage[(8 e + c) * 64 + l], so a
// wave's DMA instruction writes 1 KB contiguous and each lane reads its own 16 B (no conflicts).
// The fetch is issued before the window's cached adds and consumed after them, so the HBM/L2
// latency hides behind ~2.6k VALU instructions and no VGPR holds the entry meanwhile.
typedef __attribute__((address_space(1))) void nwc_gvoid;
typedef __attribute__((address_space(3))) void nwc_lvoid;
// One entry per stage: an 8 KB stage per wave; the second entry of a window is fetched after
// the first one has been read (it lands during the first Niels add).  Measured +1.5 % verifies/s
// over a 16 KB two-entry stage (5 interleaved A/B pairs on two boxes, profiles/r02/experiments.md),
// at the same occupancy (VGPR-bound to 2 waves per SIMD); a non-temporal cache policy for the DMA
// measured -0.9 % (profiles/r03/experiments.md).
constexpr int STAGE_U4_PER_WAVE = 8 * 64;
__device__ __forceinline__ void stage_fetch(uint4* stage, int e, const ge_niels_pad* src) {
  const uint4* g = reinterpret_cast<const uint4*>(src);
  _Pragma("unroll") for (int c = 0; c < 8; ++c)
    __builtin_amdgcn_global_load_lds((nwc_gvoid*)(g + c), (nwc_lvoid*)(stage + (8 * e + c) * 64), 16, 0, 0);
}
__device__ __forceinline__ ge_niels stage_read(const uint4* stage, int e) {
  const int lane = threadIdx.x & 63;
  union { uint4 q[8]; ge_niels_pad p; } u;
  _Pragma("unroll") for (int c = 0; c < 8; ++c) u.q[c] = stage[(8 * e + c) * 64 + lane];
  return u.p.n;
}
__device__ __forceinline__ void stage_wait() {
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the DMA has landed in LDS
}

// Smallest W in [33, 37] with x < 2^(4W-1) for all lanes (bits = bit length per lane); 38 if none.
__device__ __forceinline__ int wave_windows(int bits) {
  int W = HALF_WINDOWS_MIN;
  _Pragma("unroll") for (int k = HALF_WINDOWS_MIN; k <= HALF_WINDOWS_MAX; ++k)
    W += __any(bits > 4 * k - 1) ? 1 : 0;
  return W;
}

// A cached entry (Y+X, Y-X, Z, 2dT) as a completed point: (2X : 2Y : 2Z : 2Z) -- the ladder's first
// window starts from its first entry instead of adding it to the identity (one add saved).
__device__ __forceinline__ ge_p1p1 ge_cached_to_p1p1(const ge_cached& c) {
  ge_p1p1 r;
  r.X = fe_sub(c.YpX, c.YmX);
  r.Y = fe_add(c.YpX, c.YmX);
  r.Z = fe_add(c.Z, c.Z);
  r.T = r.Z;
  return r;
}

// four doublings of t (t in, t out), (X:Y:Z) only
__device__ __forceinline__ void ladder_dbl4(ge_p1p1& t) {
  ge_p2 p2 = ge_p1p1_to_p2_acc(t);
#pragma unroll 1
  for (int j = 0; j < 3; ++j) { t = ge_p2_dbl(p2); p2 = ge_p1p1_to_p2_acc(t); }
  t = ge_p2_dbl(p2);
}

// Basepoint digits of window w: settle pending loads, then DMA the entries into the wave's stage.
// Returns the number of entries fetched (0, 1 or 2).
__device__ __forceinline__ int base_fetch(int w, BaseDigits bd, i32& d0, i32& d1,
                                          const ge_niels_pad* T24, uint4* stage) {
  const int nb = base_window_digits(w);
  if (nb) {
    const int i = w / 6;
    d0 = bd.p[i * 256];
    // settle the A/R entry loads first (they landed during the doublings), so no wait placed
    // for them below also has to wait for the DMA
    stage_wait();
    stage_fetch(stage, 0, T24 + (d0 < 0 ? -d0 : d0));
    if (nb == 2) d1 = bd.p[(BD_HI + i) * 256];
  }
  return nb;
}
__device__ __forceinline__ void base_adds(ge_p1p1& t, int nb, i32 d0, i32 d1, uint4* stage,
                                          const ge_niels_pad* T24) {
  if (nb) {
    stage_wait();
#pragma unroll 1
    for (int side = 0; side < nb; ++side) {
      const i32 dd_ = side ? d1 : d0;
      const ge_niels e = stage_read(stage, 0);
      if (side + 1 < nb) {
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): entry 0 is in VGPRs before the slot is reused
        stage_fetch(stage, 0, T24 + B24_ENTRIES + (d1 < 0 ? -d1 : d1));
      }
      t = ge_add_niels(ge_p1p1_to_p3_acc(t), ge_niels_cneg(e, dd_ < 0));
      if (side + 1 < nb) stage_wait();
    }
  }
}

__device__ __forceinline__ ge_p2 half_scalarmult(const LaneTable& ta, const LaneTable& tr, Digits16 cd, Digits16 dd,
                                                 BaseDigits bd, const ge_niels_pad* T24,
                                                 uint4* stage, int W) {
  // Code-size discipline: the window body holds ONE doubling and ONE Niels add (rolled loops) and
  // two cached adds, so the hot loop stays inside the instruction cache.
  i32 da = cd.top, dr = dd.top;   // top digits are >= 0
  // No entry is held across the doublings (holding the next window's entries through them, as
  // rounds 1-2 did, kept 80 VGPRs live and spilled): each is gathered inside its add; the digit
  // strings are parked in LDS (BaseDigits), so the loop carries only the accumulator and a few
  // scalars
  park16(bd, BD_C, cd);
  park16(bd, BD_D, dd);
  ge_p1p1 t = ge_cached_to_p1p1(lt_first(ta, da));
#pragma unroll 1
  for (int w = W - 1; w >= 0; --w) {
    i32 d0 = 0, d1 = 0;
    // the window's first basepoint entry lands during the doublings; the A/R gathers issued
    // after it then never wait on the DMA (vmcnt counts in order)
    const int nb = base_fetch(w, bd, d0, d1, T24, stage);
    if (w != W - 1) {
      ladder_dbl4(t);
      da = digit16(bd, BD_C, w, W);
      t = add_lt(t, ta, da < 0 ? -da : da, da < 0);
      dr = digit16(bd, BD_D, w, W);
    }
    t = add_lt(t, tr, dr < 0 ? -dr : dr, dr < 0);
    base_adds(t, nb, d0, d1, stage, T24);
  }
  return ge_p1p1_to_p2(t);
}

// The same ladder over digit strings already parked in LDS (BD_C, BD_D; top digits passed in).
__device__ __forceinline__ ge_p2 half_scalarmult_parked(const LaneTable& ta, const LaneTable& tr, i32 c_top, i32 d_top,
                                                        BaseDigits bd, const ge_niels_pad* T24, uint4* stage, int W) {
  i32 da = c_top, dr = d_top;   // top digits are >= 0
  ge_p1p1 t = ge_cached_to_p1p1(lt_first(ta, da));
#pragma unroll 1
  for (int w = W - 1; w >= 0; --w) {
    i32 d0 = 0, d1 = 0;
    const int nb = base_fetch(w, bd, d0, d1, T24, stage);
    if (w != W - 1) {
      ladder_dbl4(t);
      da = digit16(bd, BD_C, w, W);
      t = add_lt(t, ta, da < 0 ? -da : da, da < 0);
      dr = digit16(bd, BD_D, w, W);
    }
    t = add_lt(t, tr, dr < 0 ? -dr : dr, dr < 0);
    base_adds(t, nb, d0, d1, stage, T24);
  }
  return ge_p1p1_to_p2(t);
}

// Half-size ladder with a cached key: Q = eB*B + c'*(-A) + d*(-R) where the A term uses the key's
// radix-256 Niels table (one add at every even window, no per-equation table or decompression).
// ca: radix-256 digits of |c| starting at window (W-1) & ~1; c_neg flips every A entry.
__device__ __forceinline__ ge_p2 half_scalarmult_cached(const LaneTable& tr, Digits16 dd, Digits256 ca, bool c_neg,
                                                        const ge_niels* key_tab, BaseDigits bd,
                                                        const ge_niels_pad* T24, uint4* stage, int W) {
  i32 dr = dd.top;   // >= 0
  ge_cached er = tr.load(dr);
  ge_p1p1 t = ge_cached_to_p1p1(lt_first(tr, dr));
  i32 dA = next256(ca);
  ge_niels ean = key_tab[dA < 0 ? -dA : dA];
#pragma unroll 1
  for (int w = W - 1; w >= 0; --w) {
    if (w != W - 1) ladder_dbl4(t);
    i32 d0 = 0, d1 = 0;
    const int nb = base_fetch(w, bd, d0, d1, T24, stage);
    if (w != W - 1) t = ge_add_cached(ge_p1p1_to_p3_acc(t), ge_cached_cneg(er, dr < 0));
    if ((w & 1) == 0) t = ge_add_niels(ge_p1p1_to_p3_acc(t), ge_niels_cneg(ean, (dA < 0) != c_neg));
    base_adds(t, nb, d0, d1, stage, T24);
    if (w > 0) {
      dr = next16(dd);
      er = tr.load(dr < 0 ? -dr : dr);
      if ((w & 1) == 0) {
        dA = next256(ca);
        ean = key_tab[dA < 0 ? -dA : dA];
      }
    }
  }
  return ge_p1p1_to_p2(t);
}

// One decompression per call (a noinline body shared by every call site: I-cache).  The two
// points of an equation are decoded one after the other; each field op inside is already 10
// independent multiply-accumulate chains (fe_asm.h), and interleaving two exponentiations
// doubled the live field elements past the 2-waves/SIMD register budget.
// K separates the copy called by the half-size k_verify kernels (K = 1) from the others, so the
// register budget of their launch bounds reaches it (a callee shared with lower-occupancy
// kernels would be allocated for the most permissive caller).
template <int K>
__device__ __noinline__ void decompress_k(ge_p3 out[1], const u32* a, u32 ycanon[1][8], bool ok[1]) {
  const u32* const w[1] = {a};
  ge_decompressN<1>(out, w, ycanon, ok);
}
__device__ __forceinline__ void decompress_one(ge_p3 out[1], const u32* a, u32 ycanon[1][8], bool ok[1]) {
  decompress_k<0>(out, a, ycanon, ok);
}

// k = SHA-512(R || A || M) mod l over the raw input bytes (one block: 96 bytes + padding)
__device__ __forceinline__ void challenge(const u32 rw[8], const u32 aw[8], const u32 mw[8], u32 kw[8]) {
  uint64_t w[16];
  _Pragma("unroll") for (int i = 0; i < 4; ++i) {
    w[i] = be64_from_le32(rw[2 * i], rw[2 * i + 1]);
    w[4 + i] = be64_from_le32(aw[2 * i], aw[2 * i + 1]);
    w[8 + i] = be64_from_le32(mw[2 * i], mw[2 * i + 1]);
  }
  w[12] = 0x8000000000000000ULL; w[13] = 0; w[14] = 0; w[15] = 96 * 8;
  uint64_t st[8];
  sha512_init_state(st);
  sha512_compress(st, w);
  u32 hw[16];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    hw[2 * i] = __builtin_bswap32((u32)(st[i] >> 32));
    hw[2 * i + 1] = __builtin_bswap32((u32)st[i]);
  }
  sc_reduce512(hw, kw);
}

// Shared prologue: parse, decode, small-order flag, challenge.
struct Prologue {
  ge_p3 A, R;
  u32 kw[8], sw[8];
  bool ok;   // s < l, A and R decode, and (strict) neither is small-order
};
template <int K = 0>
__device__ __forceinline__ void prologue(Prologue& p, const u32 mw[8], const u32 aw[8], const u32 sigw[16],
                                         bool strict) {
  u32 rw[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) { rw[i] = sigw[i]; p.sw[i] = sigw[8 + i]; }
  const bool s_ok = sc_lt_l(p.sw);
  u32 ya[1][8], yr[1][8];
  bool oka[1], okr[1];
  decompress_k<K>(&p.A, aw, ya, oka);
  decompress_k<K>(&p.R, rw, yr, okr);
  const bool small = strict && (ycanon_is_small_order(ya[0]) || ycanon_is_small_order(yr[0]));
  p.ok = s_ok && oka[0] && okr[0] && !small;
  challenge(rw, aw, mw, p.kw);
}

// Full-length equation: R' = k(-A) + sB == R.
__device__ bool verify_full(const u32 mw[8], const u32 aw[8], const u32 sigw[16], bool strict, const ge_niels* sB,
                            const LaneTable& tab) {
  Prologue p;
  prologue(p, mw, aw, sigw, strict);
  build_table(tab, ge_p3_neg(p.A));
  u32 kd[8], sd[8];
  sc_recode_radix16(p.kw, kd);
  sc_recode_radix256(p.sw, sd);
  const ge_p2 rp = double_scalarmult(tab, kd, sd, sB);
  const bool eq = fe_is_zero(fe_sub(rp.X, fe_mul(p.R.X, rp.Z))) && fe_is_zero(fe_sub(rp.Y, fe_mul(p.R.Y, rp.Z)));
  return p.ok && eq;
}

// e_B = d * s mod l, split at 2^141 into radix-2^24 digit queues (el, eh)
// eb = d s mod l (d < 2^160)
__device__ __forceinline__ void ds_mod_l(const u32 d[5], const u32 s[8], u32 eb[8]) {
  u32 prod[16];
  _Pragma("unroll") for (int i = 0; i < 16; ++i) prod[i] = 0;
  _Pragma("unroll") for (int x = 0; x < 5; ++x) {
    u64 carry = 0;
    _Pragma("unroll") for (int y = 0; y < 8; ++y) {
      const u64 tt = (u64)d[x] * s[y] + prod[x + y] + carry;
      prod[x + y] = (u32)tt;
      carry = tt >> 32;
    }
    prod[x + 8] = (u32)carry;
  }
  sc_reduce512(prod, eb);
}
__device__ __forceinline__ void base_digits(const u32 d[5], const u32 s[8], Digits24& el, Digits24& eh) {
  u32 eb[8];
  ds_mod_l(d, s, eb);
  constexpr int SH = B24_SPLIT_BITS - 128;
  u32 lo[5], hi[5];
  _Pragma("unroll") for (int i = 0; i < 4; ++i) lo[i] = eb[i];
  lo[4] = eb[4] & ((1u << SH) - 1u);
  _Pragma("unroll") for (int i = 0; i < 4; ++i) hi[i] = (eb[4 + i] >> SH) | (i + 5 < 8 ? eb[5 + i] << (32 - SH) : 0u);
  hi[4] = 0;
  el = recode24<B24_LO_DIGITS>(lo);
  eh = recode24<B24_HI_DIGITS>(hi);
}

// Half-size equation: [d]e = (d s mod l) B - c A - d R == O  (lattice.h).  Sets `fallback`
// when the reduction failed; the verdict is then decided by verify_full in k_verify_fallback.
// When every lane of the wave has its key in the committee cache (wave-uniform test), A comes
// from the cache: no decompression of A, no per-equation A table, 18 Niels adds for the A term.
template <bool CACHE>
__device__ __forceinline__ bool verify_half(const u32 mw[8], const u32 aw[8], const u32 sigw[16], bool strict, const ge_niels_pad* T24,
                            uint4* stage, BaseDigits bd, const LaneTable& ta, const LaneTable& tr,
                            const Committee& cm, bool& fallback, int force_w) {
  const int key = CACHE ? committee_lookup(cm, aw) : -1;
  if (CACHE && __all(key >= 0)) {
    u32 rw[8], sw[8];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { rw[i] = sigw[i]; sw[i] = sigw[8 + i]; }
    const bool s_ok = sc_lt_l(sw);
    ge_p3 R[1];
    u32 yr[1][8];
    bool r_ok[1];
    decompress_k<1>(R, rw, yr, r_ok);
    const u32 fl = cm.flags[key];
    const bool small = strict && ycanon_is_small_order(yr[0]);
    const bool ok = s_ok && key_flags_ok(fl, strict) && r_ok[0] && !small;
    u32 kw[8];
    challenge(rw, aw, mw, kw);
    const lat::HalfScalars h = lat::reduce(kw);
    // odd W: the top radix-256 digit of |c| (window W-1) is then < 2^3 + 1, never 128
    const int W = max(wave_windows(h.ok ? h.bits : 0), min(force_w, HALF_WINDOWS_MAX)) | 1;
    fallback = !h.ok;
    {
      Digits24 el, eh;
      base_digits(h.d, sw, el, eh);
      base_digits_park(bd, el, eh);
    }
    const Digits16 dd = recode16(h.d, W);
    const Digits256 ca = recode256(h.c, ((W - 1) >> 1) + 1);
    build_table(tr, ge_p3_neg(R[0]));
    const ge_p2 q = half_scalarmult_cached(tr, dd, ca, h.c_neg, cm.tables + (size_t)key * 129, bd, T24, stage, W);
    const bool ident = fe_is_zero(q.X) && fe_is_zero(fe_sub(q.Y, q.Z));
    return ok && ident && h.ok;
  }
  Prologue p;
  prologue<1>(p, mw, aw, sigw, strict);
  const lat::HalfScalars h = lat::reduce(p.kw);
  const int W = max(wave_windows(h.ok ? h.bits : 0), min(force_w, HALF_WINDOWS_MAX));
  fallback = !h.ok;
  {
    Digits24 el, eh;
    base_digits(h.d, p.sw, el, eh);
    base_digits_park(bd, el, eh);
  }
  const Digits16 cd = recode16(h.c, W), dd = recode16(h.d, W);
  // -c A = |c| * (c < 0 ? A : -A);  -d R = d * (-R)
  build_table(ta, h.c_neg ? p.A : ge_p3_neg(p.A));
  build_table(tr, ge_p3_neg(p.R));
  const ge_p2 q = half_scalarmult(ta, tr, cd, dd, bd, T24, stage, W);
  const bool ident = fe_is_zero(q.X) && fe_is_zero(fe_sub(q.Y, q.Z));
  return p.ok && ident && h.ok;
}

// ------------------------------------------------------------------------------- verify
// n equations; equation i uses msgs[32 * (msg_index ? msg_index[i] : i * msg_stride)], pks[32 i],
// sigs[64 i] (msg_stride 0 broadcasts one digest: Signature::verify_batch, crypto/src/lib.rs:214).
// out_bits[i / 64] bit (i % 64) = verdict.  Persistent grid: block b processes 256-lane tiles
// b, b + gridDim.x, ...; lane slot (blockIdx.x * 256 + threadIdx.x) of `scratch` holds its two
// tables.  half != 0: half-size equations; lanes whose reduction fails are appended to
// fb_list (fb_count) and decided by k_verify_fallback.
struct VerifyArgs {
  const uint8_t* msgs;
  const uint32_t* msg_index;
  uint64_t msg_stride;
  const uint8_t* pks;
  const uint8_t* sigs;
  uint64_t* out_bits;
  uint64_t n;
  int strict;
  const ge_niels* base_table;   // 2 x 129 entries (radix 256; full-length ladder)
  const ge_niels_pad* base24;   // 2 x B24_ENTRIES entries (radix 2^24; half-size ladder)
  uint8_t* scratch;             // 2 * TAB_BYTES_PER_LANE per lane slot
  uint32_t* fb_list;
  uint32_t* fb_count;
  uint32_t force_fb_every;      // test hook: route equations i % every == 0 to the fallback (0 = off)
  Committee committee;          // n == 0: no cache
  uint32_t force_windows;       // test hook: run the half-size ladder with at least this many windows (0 = off)
  uint64_t* stamps;             // k_verify<.., STAMP>: per wave {memtime, realtime} at entry and exit
};
// Extra arguments of the comb path (kept out of VerifyArgs so the headline kernel's argument
// block and register allocation do not change).
//   list mode (k_verify<.., LIST>): process equations list[0 .. *count) and OR their verdict bits
//   into out_bits;  k_verify_comb: appends equations whose key is not cached to list / count.
struct CombArgs {
  uint32_t* list;
  uint32_t* count;
  const ge_niels_pad* comb_base;   // radix-256 basepoint comb (COMB_PER_KEY entries; latency kernel)
  const ge_niels_pad* comb16;      // radix-2^16 basepoint comb (COMB16_TOTAL entries; k_verify_comb)
  uint8_t* vbytes;                 // latency kernel, host-mapped: per equation bit0 = valid, bit1 = key
                                   // missing (plain byte stores; nullptr = verdict words + count)
  uint32_t list_base;              // added to the equation index a comb kernel lists (a call-wide list
                                   // over consecutive launches, nwc_api.hip LV_DEFER_LIST)
};

__device__ __forceinline__ void load_inputs(const VerifyArgs& a, uint64_t i, u32 mw[8], u32 aw[8], u32 sgw[16]) {
  const uint64_t mi = a.msg_index ? (uint64_t)a.msg_index[i] : i * a.msg_stride;
  load_words8(a.msgs + 32 * mi, mw);
  load_words8(a.pks + 32 * i, aw);
  load_words8(a.sigs + 64 * i, sgw);
  load_words8(a.sigs + 64 * i + 32, sgw + 8);
}

__device__ __forceinline__ void stage_base_tables(const ge_niels* src, ge_niels* sB, int count) {
  for (int i = threadIdx.x; i < count * 30; i += blockDim.x)
    reinterpret_cast<i32*>(sB)[i] = reinterpret_cast<const i32*>(src)[i];
  __syncthreads();
}

#ifndef NWC_VERIFY_WAVES_PER_SIMD
#define NWC_VERIFY_WAVES_PER_SIMD 2
#endif
// Persistent grid (launch_verify: NWC_VERIFY_GRID_MULT blocks per resident block slot): block b
// takes the 256-lane tiles b, b + gridDim.x, ...; lane slot (blockIdx.x * 256 + threadIdx.x) of
// `scratch` holds its two tables.  Waves taking 64-lane tiles from a counter instead measured 5 %
// slower, with the tables per resident lane or per equation alike (profiles/r05/ab_verify_sched.txt).
// STAMP (a diagnostic build, never the verdict path): every wave stores s_memtime / s_memrealtime
// at entry and exit into a.stamps, so the host reads the shader clock held under the load.
template <bool HALF, bool CACHE, bool LIST = false, bool STAMP = false>
__global__ __launch_bounds__(256, NWC_VERIFY_WAVES_PER_SIMD) void k_verify(VerifyArgs a, CombArgs ca) {
  // HALF: per-wave LDS-DMA staging of radix-2^24 basepoint entries (8 KB per wave);
  // full-length ladder: the radix-256 basepoint table (15.5 KB).
  __shared__ uint4 lds[HALF ? 4 * STAGE_U4_PER_WAVE + BASE_DIGIT_WORDS * 64 : 129 * 30 / 4];
  ge_niels* sB = reinterpret_cast<ge_niels*>(lds);
  if constexpr (!HALF) stage_base_tables(a.base_table, sB, 129);
  uint64_t t_entry = 0, r_entry = 0;
  if constexpr (STAMP) {
    t_entry = __builtin_amdgcn_s_memtime();
    r_entry = __builtin_amdgcn_s_memrealtime();
  }
  uint4* stage = lds + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * STAGE_U4_PER_WAVE;
  const BaseDigits bd{reinterpret_cast<i32*>(lds + 4 * STAGE_U4_PER_WAVE) + threadIdx.x};
  const uint64_t n = LIST ? (uint64_t)*ca.count : a.n;
  const u32 lane = threadIdx.x & 63u;
  const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t* base = a.scratch + slot * 2 * TAB_BYTES_PER_LANE;
  const LaneTable ta{reinterpret_cast<uint4*>(base)};
  const LaneTable tr{reinterpret_cast<uint4*>(base + TAB_BYTES_PER_LANE)};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t bb = (uint64_t)blockIdx.x * blockDim.x; bb < n; bb += stride) {
    const uint64_t b0 = bb + (threadIdx.x & ~63u);   // this wave's 64 equations
    const u32 tile = (u32)(b0 >> 6);
    const uint64_t idx = b0 + lane;
    const bool active = idx < n;
    const uint64_t i = LIST ? (active ? (uint64_t)ca.list[idx] : 0) : idx;
    u32 mw[8], aw[8], sgw[16];
    load_inputs(a, active ? i : 0, mw, aw, sgw);
    bool fb = false;
    bool v;
    if constexpr (HALF) v = verify_half<CACHE>(mw, aw, sgw, a.strict != 0, a.base24, stage, bd, ta, tr, a.committee, fb,
                                                 (int)a.force_windows);
    else v = verify_full(mw, aw, sgw, a.strict != 0, sB, ta);
    if (HALF && a.force_fb_every && (i % a.force_fb_every) == 0) { fb = true; v = false; }
    v = v && active;
    fb = fb && active;
    if (fb) a.fb_list[atomicAdd(a.fb_count, 1u)] = (uint32_t)i;
    if constexpr (LIST) {
      if (v) atomicOr(reinterpret_cast<unsigned long long*>(a.out_bits) + (i >> 6), 1ull << (i & 63));
    } else {
      const uint64_t ballot = __ballot(v);
      if (lane == 0 && b0 < n) a.out_bits[tile] = ballot;
    }
  }
  if constexpr (STAMP) {
    const uint64_t t_exit = __builtin_amdgcn_s_memtime();
    const uint64_t r_exit = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      uint64_t* w = a.stamps + 4 * ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
      w[0] = t_entry; w[1] = t_exit; w[2] = r_entry; w[3] = r_exit;
    }
  }
}

template __global__ void k_verify<true, false>(VerifyArgs, CombArgs);
template __global__ void k_verify<true, true>(VerifyArgs, CombArgs);
template __global__ void k_verify<false, false>(VerifyArgs, CombArgs);
template __global__ void k_verify<true, false, true>(VerifyArgs, CombArgs);
template __global__ void k_verify<true, false, false, true>(VerifyArgs, CombArgs);

// Full-length re-verification of the lanes k_verify could not reduce (rare); sets their bits.
__global__ __launch_bounds__(256) void k_verify_fallback(VerifyArgs a) {
  __shared__ ge_niels sB[129];
  const uint32_t count = *a.fb_count;
  if (count == 0) return;   // the usual case: no table staging, ~2 us
  stage_base_tables(a.base_table, sB, 129);
  const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const LaneTable ta{reinterpret_cast<uint4*>(a.scratch + slot * 2 * TAB_BYTES_PER_LANE)};
  for (uint32_t j = (uint32_t)slot; j < count; j += gridDim.x * blockDim.x) {
    const uint64_t i = a.fb_list[j];
    u32 mw[8], aw[8], sgw[16];
    load_inputs(a, i, mw, aw, sgw);
    if (verify_full(mw, aw, sgw, a.strict != 0, sB, ta))
      atomicOr(reinterpret_cast<unsigned long long*>(a.out_bits) + (i >> 6), 1ull << (i & 63));
  }
}

// ------------------------------------------------------------------------------- torsion of batch-leaf keys
// Batch-leaf equations (strict == 0) whose key is NOT in the committee cache have passed e == O
// without the key's torsion test.  A launch of n equations dedupes the keys of the equations that
// passed in a per-launch hash set (k_tors_mark; cached keys instead use their KEY_TORSION flag
// directly), tests each distinct key once (k_tors_eval: ge_has_torsion), and clears the verdict bit
// of every equation whose key has torsion (k_tors_apply).  Committees repeat keys, so the distinct
// count -- and the cost -- is the committee size, not the vote count.
// A key's torsion is a fixed property, so every evaluated key is also memoised in a per-device
// table that persists across launches (KeyMemo: open addressing on the exact 32 bytes, bounded
// probes, never evicted; a full table just stops memoising).  Verdicts do not depend on it: a
// key found there carries the flag ge_has_torsion computed for exactly those bytes.
struct KeyMemo {
  u32* keys;                // slots x 8 words
  u32* flag;                // per slot: MEMO_EMPTY, or the key's torsion bit (0 / 1)
  u32 slot_mask;
};
constexpr u32 MEMO_EMPTY = 0xFFFFFFFFu, MEMO_BUSY = 0xFFFFFFFEu;
constexpr int MEMO_MAX_PROBE = 32;
__device__ __forceinline__ int memo_lookup(const KeyMemo& m, const u32 aw[8]) {
  if (!m.keys) return -1;
  u32 h = committee_hash(aw[0], aw[1]) & m.slot_mask;
  for (int p = 0; p < MEMO_MAX_PROBE; ++p, h = (h + 1) & m.slot_mask) {
    const u32 f = m.flag[h];
    if (f == MEMO_EMPTY) return -1;
    if (f == MEMO_BUSY) continue;
    u32 d = 0;
    _Pragma("unroll") for (int k = 0; k < 8; ++k) d |= m.keys[8 * h + k] ^ aw[k];
    if (d == 0) return (int)f;
  }
  return -1;
}
__device__ __forceinline__ void memo_insert(const KeyMemo& m, const u32 aw[8], u32 torsion) {
  if (!m.keys) return;
  u32 h = committee_hash(aw[0], aw[1]) & m.slot_mask;
  for (int p = 0; p < MEMO_MAX_PROBE; ++p, h = (h + 1) & m.slot_mask) {
    if (atomicCAS(&m.flag[h], MEMO_EMPTY, MEMO_BUSY) == MEMO_EMPTY) {
      _Pragma("unroll") for (int k = 0; k < 8; ++k) m.keys[8 * h + k] = aw[k];
      __threadfence();
      atomicExch(&m.flag[h], torsion);
      return;
    }
  }
}

struct TorsArgs {
  const uint8_t* pks;
  uint64_t* bits;           // the launch's verdict words
  const uint32_t* list;     // nullptr: equations 0 .. n-1; else list[0 .. *count)
  const uint32_t* count;
  uint64_t n;
  int32_t* slots;           // hash set: representative equation index, -1 = empty
  uint32_t slot_mask;
  uint32_t* uniq;           // slots that hold a distinct key
  uint32_t* nuniq;
  uint32_t* tflag;          // per slot: 1 = the key has torsion
  Committee committee;
  KeyMemo memo;
  int pre;   // 1: mark/eval run before (or beside) the verification: every equation is a candidate,
             //    k_tors_mark leaves the verdict words alone and k_tors_apply also applies the
             //    committee flags
};
__device__ __forceinline__ bool tors_candidate(const TorsArgs& t, uint64_t idx, uint64_t& i, u32 aw[8], int& key,
                                               bool need_bit = true) {
  i = t.list ? (uint64_t)t.list[idx] : idx;
  if (need_bit && !((t.bits[i >> 6] >> (i & 63)) & 1)) return false;
  load_words8(t.pks + 32 * i, aw);
  key = committee_lookup(t.committee, aw);
  return true;
}
__device__ __forceinline__ bool tors_key_eq(const uint8_t* pks, int32_t rep, const u32 aw[8]) {
  u32 w[8];
  load_words8(pks + 32 * (uint64_t)rep, w);
  u32 d = 0;
  _Pragma("unroll") for (int k = 0; k < 8; ++k) d |= w[k] ^ aw[k];
  return d == 0;
}
__global__ __launch_bounds__(256) void k_tors_mark(TorsArgs t) {
  const uint64_t N = t.list ? (uint64_t)*t.count : t.n;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < N; idx += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i;
    u32 aw[8];
    int key;
    if (!tors_candidate(t, idx, i, aw, key, !t.pre)) continue;
    const int known = key >= 0 ? (int)((t.committee.flags[key] & KEY_TORSION) != 0) : memo_lookup(t.memo, aw);
    if (known >= 0) {
      if (known && !t.pre) atomicAnd(reinterpret_cast<unsigned long long*>(t.bits) + (i >> 6), ~(1ull << (i & 63)));
      continue;
    }
    u32 h = committee_hash(aw[0], aw[1]) & t.slot_mask;
    for (;;) {   // the set holds at most half its slots: the probe ends
      int32_t cur = t.slots[h];
      if (cur < 0) {
        cur = atomicCAS(&t.slots[h], -1, (int32_t)i);
        if (cur < 0) { t.uniq[atomicAdd(t.nuniq, 1u)] = h; break; }
      }
      if (tors_key_eq(t.pks, cur, aw)) break;
      h = (h + 1) & t.slot_mask;
    }
  }
}
__global__ __launch_bounds__(256) void k_tors_eval(TorsArgs t) {
  const uint32_t N = *t.nuniq;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < N; j += gridDim.x * blockDim.x) {
    const uint32_t h = t.uniq[j];
    u32 aw[8];
    load_words8(t.pks + 32 * (uint64_t)t.slots[h], aw);
    ge_p3 A[1];
    u32 yc[1][8];
    bool ok[1];
    decompress_one(A, aw, yc, ok);
    const u32 tor = (ok[0] && ge_has_torsion(A[0])) ? 1u : 0u;
    t.tflag[h] = tor;
    if (ok[0]) memo_insert(t.memo, aw, tor);
  }
}
__global__ __launch_bounds__(256) void k_tors_apply(TorsArgs t) {
  const uint64_t N = t.list ? (uint64_t)*t.count : t.n;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < N; idx += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i;
    u32 aw[8];
    int key;
    if (!tors_candidate(t, idx, i, aw, key)) continue;
    if (key >= 0) {   // cached key: its flag (k_tors_mark applied it unless pre)
      if (t.pre && (t.committee.flags[key] & KEY_TORSION))
        atomicAnd(reinterpret_cast<unsigned long long*>(t.bits) + (i >> 6), ~(1ull << (i & 63)));
      continue;
    }
    // memoised keys (found by k_tors_mark, or memoised by k_tors_eval just now) carry their flag;
    // clearing a bit k_tors_mark already cleared is harmless
    const int known = memo_lookup(t.memo, aw);
    if (known >= 0) {
      if (known) atomicAnd(reinterpret_cast<unsigned long long*>(t.bits) + (i >> 6), ~(1ull << (i & 63)));
      continue;
    }
    // k_tors_mark inserted the key at or before the first empty slot of its probe sequence
    u32 h = committee_hash(aw[0], aw[1]) & t.slot_mask;
    int32_t rep = t.slots[h];
    while (rep >= 0 && !tors_key_eq(t.pks, rep, aw)) {
      h = (h + 1) & t.slot_mask;
      rep = t.slots[h];
    }
    // (rep < 0 cannot happen; clearing the bit then errs on the side of Err)
    if (rep < 0 || t.tflag[h]) atomicAnd(reinterpret_cast<unsigned long long*>(t.bits) + (i >> 6), ~(1ull << (i & 63)));
  }
}

// ------------------------------------------------------------------------------- committee comb verify
// Doubling-free verification for equations whose key is in the committee cache:
//   R' = s B + k (-A) = sum_w combB[w][s_w] + sum_w combA_key[w][k_w]      (64 Niels adds)
// and R' == R is decided on the compressed form: y(R') == y_R mod p and sign(x(R')) == bit 255 of
// R (any sign when x(R') = 0, since dalek decodes -0 as 0).  This is exactly dalek's decision
// "R decodes and R' == R as points": if the encodings agree, R decodes to R'; if R does not decode
// no point has its y.  Small-order R (strict) is read off the canonical y of the encoding (every
// small-order y decodes).  Compressing needs 1/Z; the lane batches the inversions of COMB_BATCH
// equations (Montgomery: one exponentiation + 3 multiplications each) -- a decompression of R, the
// alternative, is a square root and cannot be batched.
// Equations whose key is not cached go to uc_list and are verified by k_verify in list mode.
struct CombRec { fe X, Y, Z, P; u32 yr[8]; u32 meta; u32 pad[3]; };
static_assert(sizeof(CombRec) == 208, "comb record layout");
#ifndef NWC_COMB_BATCH
#define NWC_COMB_BATCH 64
#endif
constexpr int COMB_BATCH = NWC_COMB_BATCH;
constexpr size_t COMB_REC_U4 = sizeof(CombRec) / 16;
constexpr size_t COMB_BYTES_PER_LANE = COMB_BATCH * sizeof(CombRec);

// entry |d| of window w of a comb with `entries` entries per window
__device__ __forceinline__ ge_niels comb_load(const ge_niels_pad* tab, int entries, int w, i32 d) {
  const uint4* q = reinterpret_cast<const uint4*>(tab + (size_t)w * entries + (d < 0 ? -d : d));
  union { uint4 u[8]; ge_niels_pad p; } e;
  _Pragma("unroll") for (int c = 0; c < 8; ++c) e.u[c] = q[c];
  return e.p.n;
}
// Records are lane-interleaved: uint4 c of record j of lane slot l sits at
// scratch[(j * COMB_REC_U4 + c) * lanes + l], so each of a wave's 13 record stores/loads moves one
// contiguous KB (lanes = the persistent grid's lane count).
__device__ __forceinline__ void rec_store(uint4* base, size_t lanes, int j, const CombRec& r) {
  const uint4* src = reinterpret_cast<const uint4*>(&r);
  _Pragma("unroll") for (size_t c = 0; c < COMB_REC_U4; ++c) base[(j * COMB_REC_U4 + c) * lanes] = src[c];
}
__device__ __forceinline__ CombRec rec_load(const uint4* base, size_t lanes, int j) {
  CombRec r;
  uint4* dst = reinterpret_cast<uint4*>(&r);
  _Pragma("unroll") for (size_t c = 0; c < COMB_REC_U4; ++c) dst[c] = base[(j * COMB_REC_U4 + c) * lanes];
  return r;
}
// affine Niels entry as a completed point (2x : 2y : 2 : 2) -- starts the sum without an add
__device__ __forceinline__ ge_p1p1 ge_niels_to_p1p1(const ge_niels& q) {
  ge_p1p1 r;
  r.X = fe_sub(q.ypx, q.ymx);
  r.Y = fe_add(q.ypx, q.ymx);
  r.Z = fe_zero(); r.Z.v[0] = 2;
  r.T = r.Z;
  return r;
}

// s B + k (-A) with the basepoint comb (COMB16_WINDOWS windows of radix 2^NWC_BCOMB_BITS) and the
// key's comb (radix 2^14, 19 windows): 31 additions by default -- the key's windows, then B's.  Entry i+1 is fetched
// before entry i is added, so one fetch is in flight behind every addition.
constexpr int COMB_SUM_ADDS = KeyComb::windows + COMB16_WINDOWS;   // 31 (19 key + 12 basepoint windows)
__device__ __forceinline__ ge_p2 comb_sum(const u32 sw[8], const u32 kw[8], const ge_niels_pad* TB16,
                                          const ge_niels_pad* TA) {
  u32 sd[9], kd[9];
  sc_recode_radix<NWC_BCOMB_BITS, COMB16_WINDOWS>(sw, sd);
  sc_recode_radix<KeyComb::bits, KeyComb::windows>(kw, kd);
  i32 d = digit_at<KeyComb::bits>(kd, KeyComb::windows - 1);
  ge_niels e = comb_load(TA, KeyComb::entries, KeyComb::windows - 1, d);
  ge_p1p1 t = ge_niels_to_p1p1(ge_niels_cneg(e, d < 0));
  i32 dn = digit_at<KeyComb::bits>(kd, KeyComb::windows - 2);
  ge_niels en = comb_load(TA, KeyComb::entries, KeyComb::windows - 2, dn);
#pragma unroll 1
  for (int i = 1; i < COMB_SUM_ADDS; ++i) {
    e = en;
    d = dn;
    const int nx = i + 1;   // entry to fetch: key window 21 - nx, or B window 37 - nx
    if (nx < KeyComb::windows) {
      dn = digit_at<KeyComb::bits>(kd, KeyComb::windows - 1 - nx);
      en = comb_load(TA, KeyComb::entries, KeyComb::windows - 1 - nx, dn);
    } else if (nx < COMB_SUM_ADDS) {
      dn = digit_at<NWC_BCOMB_BITS>(sd, COMB_SUM_ADDS - 1 - nx);
      en = comb_load(TB16, COMB16_ENTRIES, COMB_SUM_ADDS - 1 - nx, dn);
    }
    t = ge_add_niels(ge_p1p1_to_p3(t), ge_niels_cneg(e, d < 0));
  }
  return ge_p1p1_to_p2(t);
}

__global__ __launch_bounds__(256, 2) void k_verify_comb(VerifyArgs a, CombArgs ca) {
  const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4* recs = reinterpret_cast<uint4*>(a.scratch) + slot;
  const size_t lanes = (size_t)gridDim.x * blockDim.x;
  const Committee& cm = a.committee;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c0 = (uint64_t)blockIdx.x * blockDim.x; c0 < a.n; c0 += stride * COMB_BATCH) {
    // forward: R' of up to COMB_BATCH equations, running product of their Z
    fe P = fe_one();
    int nb = 0;
#pragma unroll 1
    for (int j = 0; j < COMB_BATCH; ++j) {
      const uint64_t b0 = c0 + (uint64_t)j * stride;
      if (b0 >= a.n) break;   // block-uniform
      const uint64_t i = b0 + threadIdx.x;
      const bool active = i < a.n;
      u32 mw[8], aw[8], sgw[16];
      load_inputs(a, active ? i : 0, mw, aw, sgw);
      const int key = committee_lookup(cm, aw);
      if (active && key < 0) ca.list[atomicAdd(ca.count, 1u)] = ca.list_base + (uint32_t)i;
      const int kk = key < 0 ? 0 : key;
      u32 rw[8], sw[8];
      _Pragma("unroll") for (int q = 0; q < 8; ++q) { rw[q] = sgw[q]; sw[q] = sgw[8 + q]; }
      CombRec r;
      fe_to_words(fe_from_words(rw), r.yr);   // y_R mod p
      const u32 fl = cm.flags[kk];
      const bool small = a.strict && ycanon_is_small_order(r.yr);
      const bool ok = active && key >= 0 && sc_lt_l(sw) && key_flags_ok(fl, a.strict != 0) && !small;
      ge_p2 q;
      if (__any(key >= 0)) {
        u32 kw[8];
        challenge(rw, aw, mw, kw);
        q = comb_sum(sw, kw, ca.comb16, cm.comb + (size_t)kk * COMB_PER_KEY);
      } else {
        // no equation of this wave has a cached key (launch keys: another committee's votes, or a
        // launch without repeated keys): skip the sum, the list-mode ladder decides them all
        q.X = fe_zero();
        q.Y = fe_one();
        q.Z = fe_one();
      }
      // Z != 0 for every sum of curve points (complete formulas); a key that does not decode has
      // an off-curve comb, whose Z must not zero the lane's batched inversion
      const bool zbad = fe_is_zero(q.Z);
      r.X = q.X; r.Y = q.Y; r.Z = fe_select(q.Z, fe_one(), zbad); r.P = P;
      r.meta = (ok && !zbad ? 1u : 0u) | ((rw[7] >> 31) << 1);
      r.pad[0] = r.pad[1] = r.pad[2] = 0;
      rec_store(recs, lanes, j, r);
      P = fe_mul(P, r.Z);
      nb = j + 1;
    }
    // one inversion for the lane's nb equations, then backwards: 1/Z_j = inv * P_{j-1}
    fe inv = fe_invert(P);
#pragma unroll 1
    for (int j = nb - 1; j >= 0; --j) {
      const CombRec r = rec_load(recs, lanes, j);
      const fe zi = fe_mul(inv, r.P);
      inv = fe_mul(inv, r.Z);
      u32 yw[8], xw[8];
      fe_to_words(fe_mul(r.Y, zi), yw);
      fe_to_words(fe_mul(r.X, zi), xw);
      u32 diff = 0, xor_ = 0;
      _Pragma("unroll") for (int q = 0; q < 8; ++q) { diff |= yw[q] ^ r.yr[q]; xor_ |= xw[q]; }
      const bool sign_ok = xor_ == 0 || (xw[0] & 1) == ((r.meta >> 1) & 1);
      const bool v = (r.meta & 1) && diff == 0 && sign_ok;
      const uint64_t b0 = c0 + (uint64_t)j * stride;
      const uint64_t ballot = __ballot(v);
      if ((threadIdx.x & 63) == 0 && b0 + (threadIdx.x & ~63u) < a.n) a.out_bits[(b0 + threadIdx.x) >> 6] = ballot;
    }
  }
}

// ------------------------------------------------------------------------------- comb verify, sign deferred
// k_verify_comb amortises each lane's inversion (~31k VALU instructions, 254 squarings) over the
// lane's equations of the launch.  A launch of about one resident round (the message pipeline's
// per-chunk leaf launches: ~160k votes on 131k lanes) gives a lane one or two equations, and the
// inversion then costs as much as the rest of the equation: such launches ran at ~370 M votes/s
// against ~640 M in a long launch.  Split the decision instead:
//   k_verify_comb_y: R' = sB + k(-A) by the combs (as k_verify_comb), and y(R') == y_R tested
//     projectively, Y == y_R Z (mod p): no inversion.  Equation i's X and Z (canonical words) and
//     a pending bit (key cached, flags, s < l, not small-order, Y test) go to record i of SignRecs
//     (the caller offsets the arrays).  No verdict word is written.
//   k_comb_sign: later, once over many votes, the sign of x(R') = X/Z against R's sign bit, with
//     one inversion per lane over ~8 votes (Montgomery's trick along the lane's strided votes);
//     ORs pending && sign ok into the verdict words of its range, which the caller zeroed (the
//     uncached keys' list passes OR theirs in too, before or after).
// Same decision as k_verify_comb: y(R') == y_R mod p and sign(x(R')) == bit 255 of R (any sign
// when x(R') = 0).
struct SignRecs {
  u32* x;      // 8 words per vote: X of R' (canonical)
  u32* z;      // 8 words per vote: Z of R' (canonical; 1 when Z == 0)
  u32* p;      // 8 words per vote: k_comb_sign's running product before the vote
  u32* meta;   // bit 0 pending, bit 1 R's sign bit
};

// (bodies over blocks [blk, nblk) of the grid: k_verify_comb_y_sign runs both in one launch)
__device__ __forceinline__ void comb_y_body(const VerifyArgs& a, const CombArgs& ca, const SignRecs& sr, uint32_t blk,
                                            uint32_t nblk) {
  const Committee& cm = a.committee;
  const uint64_t stride = (uint64_t)nblk * blockDim.x;
  for (uint64_t b0 = (uint64_t)blk * blockDim.x; b0 < a.n; b0 += stride) {   // block-uniform
    const uint64_t i = b0 + threadIdx.x;
    const bool active = i < a.n;
    u32 mw[8], aw[8], sgw[16];
    load_inputs(a, active ? i : 0, mw, aw, sgw);
    const int key = committee_lookup(cm, aw);
    // (no list: the caller does not need uncached equations decided, their verdict stays 0)
    if (active && key < 0 && ca.list) ca.list[atomicAdd(ca.count, 1u)] = ca.list_base + (uint32_t)i;
    const int kk = key < 0 ? 0 : key;
    u32 rw[8], sw[8];
    _Pragma("unroll") for (int q = 0; q < 8; ++q) { rw[q] = sgw[q]; sw[q] = sgw[8 + q]; }
    const fe yr = fe_from_words(rw);   // y_R mod p (bit 255 ignored)
    u32 yw[8];
    fe_to_words(yr, yw);
    const u32 fl = cm.flags[kk];
    const bool small = a.strict && ycanon_is_small_order(yw);
    const bool ok = active && key >= 0 && sc_lt_l(sw) && key_flags_ok(fl, a.strict != 0) && !small;
    ge_p2 q;
    if (__any(key >= 0)) {
      u32 kw[8];
      challenge(rw, aw, mw, kw);
      q = comb_sum(sw, kw, ca.comb16, cm.comb + (size_t)kk * COMB_PER_KEY);
    } else {
      q.X = fe_zero();
      q.Y = fe_one();
      q.Z = fe_one();
    }
    const bool zbad = fe_is_zero(q.Z);   // an undecodable key's off-curve comb (see k_verify_comb)
    const bool ymatch = fe_is_zero(fe_sub(fe_mul(yr, q.Z), q.Y));
    u32 xw[8], zw[8];
    fe_to_words(q.X, xw);
    fe_to_words(fe_select(q.Z, fe_one(), zbad), zw);
    if (active) {
      const uint64_t v = i;
      uint4* xd = reinterpret_cast<uint4*>(sr.x + 8 * v);
      uint4* zd = reinterpret_cast<uint4*>(sr.z + 8 * v);
      xd[0] = make_uint4(xw[0], xw[1], xw[2], xw[3]);
      xd[1] = make_uint4(xw[4], xw[5], xw[6], xw[7]);
      zd[0] = make_uint4(zw[0], zw[1], zw[2], zw[3]);
      zd[1] = make_uint4(zw[4], zw[5], zw[6], zw[7]);
      sr.meta[v] = (ok && !zbad && ymatch ? 1u : 0u) | ((rw[7] >> 31) << 1);
    }
  }
}

__global__ __launch_bounds__(256, 2) void k_verify_comb_y(VerifyArgs a, CombArgs ca, SignRecs sr) {
  comb_y_body(a, ca, sr, blockIdx.x, gridDim.x);
}

__device__ __forceinline__ fe load_fe_words(const u32* p) {
  const uint4* s = reinterpret_cast<const uint4*>(p);
  const uint4 u0 = s[0], u1 = s[1];
  const u32 w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
  return fe_from_words(w);
}

// Votes [v0, v0 + n) (v0 a multiple of 64; the lane count a multiple of 64), vote v's record at
// index v of sr (the caller offsets the arrays): lane l takes votes v0 + l + j * lanes, so a
// wave's step j is one aligned verdict word.
__device__ __forceinline__ void comb_sign_body(const SignRecs& sr, uint64_t v0, uint64_t n, uint64_t* out_bits,
                                               uint32_t blk, uint32_t nblk) {
  const uint64_t lanes = (uint64_t)nblk * blockDim.x;
  const uint64_t l = (uint64_t)blk * blockDim.x + threadIdx.x;
  const uint64_t wb = l & ~63ull;
  const uint64_t steps = wb < n ? (n - wb + lanes - 1) / lanes : 0;   // wave-uniform
  fe P = fe_one();
#pragma unroll 1
  for (uint64_t j = 0; j < steps; ++j) {
    const uint64_t idx = l + j * lanes;
    const bool active = idx < n;
    const uint64_t v = v0 + (active ? idx : 0);
    if (active) {
      u32 pw[8];
      fe_to_words(P, pw);
      uint4* pd = reinterpret_cast<uint4*>(sr.p + 8 * v);
      pd[0] = make_uint4(pw[0], pw[1], pw[2], pw[3]);
      pd[1] = make_uint4(pw[4], pw[5], pw[6], pw[7]);
    }
    const fe z = active ? load_fe_words(sr.z + 8 * v) : fe_one();
    P = fe_mul(P, z);
  }
  fe inv = fe_invert(P);
#pragma unroll 1
  for (uint64_t jj = steps; jj-- > 0;) {
    const uint64_t idx = l + jj * lanes;
    const bool active = idx < n;
    const uint64_t v = v0 + (active ? idx : 0);
    const fe pb = active ? load_fe_words(sr.p + 8 * v) : fe_one();
    const fe z = active ? load_fe_words(sr.z + 8 * v) : fe_one();
    const fe zi = fe_mul(inv, pb);
    inv = fe_mul(inv, z);
    u32 xw[8];
    fe_to_words(fe_mul(load_fe_words(sr.x + 8 * v), zi), xw);
    u32 xor_ = 0;
    _Pragma("unroll") for (int q = 0; q < 8; ++q) xor_ |= xw[q];
    const u32 m = sr.meta[v];
    const bool sign_ok = xor_ == 0 || (xw[0] & 1) == ((m >> 1) & 1);
    const uint64_t ballot = __ballot(active && (m & 1) && sign_ok);
    if ((threadIdx.x & 63) == 0) out_bits[(v0 + wb + jj * lanes) >> 6] |= ballot;   // the word is this wave's
  }
}

__global__ __launch_bounds__(256) void k_comb_sign(SignRecs sr, uint64_t v0, uint64_t n, uint64_t* out_bits) {
  comb_sign_body(sr, v0, n, out_bits, blockIdx.x, gridDim.x);
}

// One launch of both: blocks [0, sign_blocks) run the previous launch's sign tests (latency-bound:
// one inversion per lane), the rest this launch's comb sums, so the sign pass's chain hides behind
// the sums instead of standing alone on the leaf stream.
struct SignPass {
  SignRecs rec;   // the previous launch's records (vote v at index v)
  uint64_t v0, n;
  uint64_t* out_bits;
  uint32_t blocks;
};
__global__ __launch_bounds__(256, 2) void k_verify_comb_y_sign(VerifyArgs a, CombArgs ca, SignRecs sr, SignPass sp) {
  if (blockIdx.x < sp.blocks)
    comb_sign_body(sp.rec, sp.v0, sp.n, sp.out_bits, blockIdx.x, sp.blocks);
  else
    comb_y_body(a, ca, sr, blockIdx.x - sp.blocks, gridDim.x - sp.blocks);
}

// ------------------------------------------------------------------------------- committee latency
// Latency form of the comb path for small batches (a certificate's votes, BASELINE cfg 1): one
// equation per 128-thread block.  Wave 0 sums the 64 comb entries of sB + k(-A) with one entry per
// lane and a 6-level butterfly (every lane ends with the sum); wave 1 decompresses R meanwhile.
// The critical path is one square root (~31k dependent VALU instructions) instead of a lane's whole
// verification.  Verdict: R decodes, R' == R projectively, plus the same s / key / small-order flags
// as k_verify_comb.  Bits are OR-ed into out_bits (zeroed by the caller).
__device__ __forceinline__ i32 digit256_at(const u32 d[8], int w) {
  u32 word = d[0];
  _Pragma("unroll") for (int q = 1; q < 8; ++q) word = (q == (w >> 2)) ? d[q] : word;
  return (i32)((word >> (8 * (w & 3))) & 255u) - 128;
}
__device__ __forceinline__ ge_p3 shfl_xor_p3(const ge_p3& p, int mask) {
  ge_p3 r;
  const i32* src = reinterpret_cast<const i32*>(&p);
  i32* dst = reinterpret_cast<i32*>(&r);
  _Pragma("unroll") for (int q = 0; q < 40; ++q) dst[q] = __shfl_xor(src[q], mask, 64);
  return r;
}

// R of the latency kernel: dalek's decompression (ge_decompress_prep / _finish) with every field
// operation on the dependent chain limb-sliced; returns the affine x, y (Z = 1) as one element per
// lane, the decode flag and the canonical y.
__device__ __forceinline__ void decompress_sliced(const u32 w[8], fe& X, fe& Y, u32 ycanon[8], bool& ok) {
  const fe yl = fe_from_words(w);
  const fes y = fes_from_fe(yl);
  const fes yy = fes_sq(y);
  const fes u = fes_add_small(yy, -1);
  const fes v = fes_add_small(fes_mul(yy, fes_from_fe(FE_D)), 1);
  const fes v3 = fes_mul(fes_sq(v), v);
  const fes v7 = fes_mul(fes_sq(v3), v);
  const fes b = fes_pow22523(fes_mul(u, v7));
  fes r = fes_mul(fes_mul(u, v3), b);                 // u v^3 (u v^7)^((p-5)/8)
  const fes check = fes_mul(v, fes_sq(r));            // v r^2
  const bool correct = fe_is_zero(fe_from_fes(fes_sub(check, u)));
  const bool flipped = fe_is_zero(fe_from_fes(fes_add(check, u)));
  const bool flipped_i = fe_is_zero(fe_from_fes(fes_add(check, fes_mul(u, fes_from_fe(FE_SQRTM1)))));
  const fes ri = fes_mul(r, fes_from_fe(FE_SQRTM1));   // no branch: DPP must see every lane of the row
  r.v = (flipped || flipped_i) ? ri.v : r.v;
  fe rl = fe_from_fes(r);
  rl = fe_select(rl, fe_neg(rl), fe_is_negative(rl));
  X = fe_select(rl, fe_neg(rl), (w[7] >> 31) & 1);
  Y = fe_tighten(yl);
  fe_to_words(yl, ycanon);
  ok = correct || flipped;
}

// Small launches (the first-sight keys of a certificate): one wave per distinct key, its
// decompression and l*A both limb-sliced (ge_sliced.h): ~160 us per key instead of ~0.8 ms on one
// lane (tools/microbench/sliced_points.hip).  Same flags and memo as k_tors_eval.
__global__ __launch_bounds__(64) void k_tors_eval_sliced(TorsArgs t) {
  const uint32_t N = *t.nuniq;
  for (uint32_t j = blockIdx.x; j < N; j += gridDim.x) {   // block-uniform: one key per wave
    const uint32_t h = t.uniq[j];
    u32 aw[8];
    load_words8(t.pks + 32 * (uint64_t)t.slots[h], aw);
    fe X, Y;
    u32 yc[8];
    bool ok;
    decompress_sliced(aw, X, Y, yc, ok);
    const bool tor = gs_has_torsion(gs_from_affine(X, Y), SC_L);
    if (threadIdx.x == 0) {
      t.tflag[h] = (ok && tor) ? 1u : 0u;
      if (ok) memo_insert(t.memo, aw, tor ? 1u : 0u);
    }
  }
}

// ---- first-sight small batches: one equation per block, every point operation limb-sliced ----
// k_verify_cold decides the same half-size equation as verify_half (lattice.h), for calls whose
// keys no cache holds (a certificate of first-sight keys), one 4-wave block per equation with
// every point operation limb-sliced (ge_sliced.h: two layers of ~0.19 us per doubling or addition
// instead of a ~1,000-instruction serial step).  Phase 1: wave 0 runs the scalar work (s < l, the
// challenge, the lattice reduction, d s mod l, the digit strings) on all its lanes, waves 1 and 2
// decompress A and R; wave 3 (batch leaf) starts u([2^252] A) from A's y at once.  Phase 2: wave 0
// the -d R share of the ladder, wave 1 the -c A share, wave 2 (batch leaf) [l - 2^252] A, wave 3
// [d s mod l] B from the basepoint comb; wave 1 adds the shares and decides.  Tables live in LDS
// as 40 limbs per entry (a row-0 lane k < 10 stores limb k of each coordinate; every lane reads
// its own limb back).
struct ColdShared {
  i32 tab[3][TAB_ENTRIES][40];   // [0] multiples of +-A (sign of c), [1] of -R, [2] of A; (YpX, YmX, Z, T2d)
  i32 ax[10], ay[10], rx[10], ry[10];
  Digits16 cd, dd;
  u32 bs[8];          // d s mod l: the basepoint's scalar
  int W, c_neg, lat_ok, s_ok, a_ok, r_ok, a_small, r_small;
  i32 rsum[40];       // wave 0's share of the ladder (the -d R terms), cached
  i32 bsum[40];       // wave 3's [d s mod l] B (basepoint comb, no doublings), cached
  i32 dq[3][10];      // batch leaf: [l - 2^252] A (wave 2), projective Edwards
  i32 tu[2][10];      // batch leaf: u([2^252] A) (wave 3), projective Montgomery (U : W)
  int ready;          // waves 0-2 done with the scalars and the decompressions
};
__device__ __forceinline__ void cold_store(i32* e, const gs_cached& c) {
  const int lane = threadIdx.x & 63;
  if (lane < 10) { e[lane] = c.YpX.v; e[10 + lane] = c.YmX.v; e[20 + lane] = c.Z.v; e[30 + lane] = c.T2d.v; }
}
// entry e of a table as a cached point; neg: the entry of the negated point (Y+X <-> Y-X, -2dT)
__device__ __forceinline__ gs_cached cold_load(const i32* e, bool neg) {
  const int k = fes_lane();
  const bool live = k < 10;
  const int kk = live ? k : 0;
  gs_cached c;
  const i32 ypx = e[kk], ymx = e[10 + kk];
  c.YpX.v = live ? (neg ? ymx : ypx) : 0;
  c.YmX.v = live ? (neg ? ypx : ymx) : 0;
  c.Z.v = live ? e[20 + kk] : 0;
  c.T2d.v = live ? (neg ? -e[30 + kk] : e[30 + kk]) : 0;
  return c;
}
// a radix-2^24 basepoint entry (affine Niels, HBM) as a cached point with Z = 1, each lane its limb
__device__ __forceinline__ gs_cached cold_base_entry(const ge_niels_pad* T, i32 d) {
  const i32* e = reinterpret_cast<const i32*>(T + (d < 0 ? -d : d));
  const int k = fes_lane();
  const bool live = k < 10, neg = d < 0;
  const int kk = live ? k : 0;
  const i32 ypx = e[kk], ymx = e[10 + kk], t = e[20 + kk];
  gs_cached c;
  c.YpX.v = live ? (neg ? ymx : ypx) : 0;
  c.YmX.v = live ? (neg ? ypx : ymx) : 0;
  c.Z.v = k == 0 ? 1 : 0;
  c.T2d.v = live ? (neg ? -t : t) : 0;
  return c;
}
__device__ __forceinline__ gs_p1p1 gs_cached_to_p1p1(const gs_cached& c) {
  gs_p1p1 r;
  r.X = fes_sub(c.YpX, c.YmX);
  r.Y = fes_add(c.YpX, c.YmX);
  r.Z = fes_add(c.Z, c.Z);
  r.T = r.Z;
  return r;
}
// digit of window w (<= W - 2) of a Digits16 string (recode16's layout: nibble w + 41 - W)
__device__ __forceinline__ i32 digit16_of(const Digits16& x, int w, int W) {
  const int pos = w + 41 - W;
  u32 word = x.w[0];
  _Pragma("unroll") for (int i = 1; i < 5; ++i) word = (pos >> 3) == i ? x.w[i] : word;
  return (i32)((word >> (4 * (pos & 7))) & 15u) - 8;
}
__device__ void cold_table(i32 (*tab)[40], const gs_p3& P) {
  gs_cached id;
  id.YpX = fes_from_fe(fe_one()); id.YmX = id.YpX; id.Z = id.YpX; id.T2d.v = 0;
  cold_store(tab[0], id);
  const gs_cached p1 = gs_to_cached(P);
  cold_store(tab[1], p1);
  gs_p3 pj = gs_to_p3(gs_dbl(gs_p3_to_p2(P)));
  cold_store(tab[2], gs_to_cached(pj));
#pragma unroll 1
  for (int j = 3; j < TAB_ENTRIES; ++j) {
    pj = gs_to_p3(gs_add_cached(pj, p1));
    cold_store(tab[j], gs_to_cached(pj));
  }
}
// [m] P for the bits [lo, hi] of the 8-word constant m (left to right; bit hi must be set)
__device__ gs_p2 gs_mul_bits(const gs_p3& P, const u32 m[8], int hi, int lo) {
  const gs_cached pc = gs_to_cached(P);
  gs_p2 acc = gs_p3_to_p2(P);
#pragma unroll 1
  for (int bit = hi - 1; bit >= lo; --bit) {
    gs_p1p1 t = gs_dbl(acc);
    if ((m[bit >> 5] >> (bit & 31)) & 1u) t = gs_add_cached(gs_to_p3(t), pc);
    acc = gs_to_p2(t);
  }
  return acc;
}
// [e] B from the radix-2^22 basepoint comb (COMB16_WINDOWS entries, one addition each), cached
__device__ gs_cached cold_comb_sum(const ge_niels_pad* comb16, const u32 e[8]) {
  u32 sd[9];
  sc_recode_radix<NWC_BCOMB_BITS, COMB16_WINDOWS>(e, sd);
  i32 db = digit_at<NWC_BCOMB_BITS>(sd, COMB16_WINDOWS - 1);
  gs_p1p1 t = gs_cached_to_p1p1(cold_base_entry(comb16 + (size_t)(COMB16_WINDOWS - 1) * COMB16_ENTRIES, db));
#pragma unroll 1
  for (int w = COMB16_WINDOWS - 2; w >= 0; --w) {
    db = digit_at<NWC_BCOMB_BITS>(sd, w);
    t = gs_add_cached(gs_to_p3(t), cold_base_entry(comb16 + (size_t)w * COMB16_ENTRIES, db));
  }
  return gs_to_cached(gs_to_p3(t));
}
__device__ __forceinline__ void cold_store_p2(i32 (*q)[10], const gs_p2& p) {
  const int lane = threadIdx.x & 63;
  if (lane < 10) { q[0][lane] = p.X.v; q[1][lane] = p.Y.v; q[2][lane] = p.Z.v; }
}
// vbytes != nullptr: zero-copy launch (inputs in pinned host memory), one verdict byte per
// equation stored straight to the host like k_verify_comb_wide's (bit 7 written, bit 0 valid, bit
// 1 = the reduction failed: the host re-runs the staged path, whose fallback kernel decides it)
__global__ __launch_bounds__(256) void k_verify_cold(VerifyArgs a, const ge_niels_pad* __restrict__ comb16,
                                                    uint8_t* vbytes) {
  __shared__ ColdShared sh;
  const uint64_t i = blockIdx.x;
  if (i >= a.n) return;   // block-uniform
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool leaf = a.strict == 0;
  if (threadIdx.x == 0) sh.ready = 0;
  __syncthreads();
#define CT(tag) do {} while (0)
  u32 mw[8], aw[8], sgw[16];
  load_inputs(a, i, mw, aw, sgw);
  u32 rw[8], sw[8];
  _Pragma("unroll") for (int q = 0; q < 8; ++q) { rw[q] = sgw[q]; sw[q] = sgw[8 + q]; }
  if (wave == 3) {
    // batch leaf: the key's torsion test l A = O  <=>  u([2^252] A) = u([l - 2^252] A) (x-only, so
    // also (2^252 + l - 2^252) A = O's sign twin, which only a point of small order can meet: then
    // 2^252 A = O and the twin needs [l - 2^252] A = O, i.e. A = O -- no torsion either way).  The
    // 252 doublings start from A's y at once, beside everything else.
    if (leaf) {
      fes U, W;
      gs_xonly_dbl_n(fes_from_fe(fe_tighten(fe_from_words(aw))), 252, U, W);
      if (lane < 10) { sh.tu[0][lane] = U.v; sh.tu[1][lane] = W.v; }
    }
    CT("xonly");
    // then [d s mod l] B from the radix-2^22 basepoint comb: 12 entries, 11 additions, no
    // doublings (wave 0 has published the scalar by now in a batch leaf; a strict call waits here)
    while (__hip_atomic_load(&sh.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 3) __builtin_amdgcn_s_sleep(1);
    u32 eb[8];
    _Pragma("unroll") for (int q = 0; q < 8; ++q) eb[q] = sh.bs[q];
    cold_store(sh.bsum, cold_comb_sum(comb16, eb));
    CT("bsum");
    __syncthreads();
    return;
  }
  if (wave == 0) {
    u32 kw[8];
    challenge(rw, aw, mw, kw);
    const lat::HalfScalars h = lat::reduce(kw);
    const int W = wave_windows(h.ok ? h.bits : 0);
    u32 eb[8];
    ds_mod_l(h.d, sw, eb);
    const Digits16 cd = recode16(h.c, W), dd = recode16(h.d, W);
    if (lane == 0) {
      sh.W = W; sh.c_neg = h.c_neg; sh.lat_ok = h.ok && W <= HALF_WINDOWS_MAX; sh.s_ok = sc_lt_l(sw);
      sh.cd = cd; sh.dd = dd;
      _Pragma("unroll") for (int q = 0; q < 8; ++q) sh.bs[q] = eb[q];
    }
  } else {
    fe X, Y;
    u32 yc[8];
    bool ok;
    decompress_sliced(wave == 1 ? aw : rw, X, Y, yc, ok);
    if (lane == 0) {
      const bool so = ycanon_is_small_order(yc);
      _Pragma("unroll") for (int q = 0; q < 10; ++q) {
        if (wave == 1) { sh.ax[q] = X.v[q]; sh.ay[q] = Y.v[q]; } else { sh.rx[q] = X.v[q]; sh.ry[q] = Y.v[q]; }
      }
      if (wave == 1) { sh.a_ok = ok; sh.a_small = so; } else { sh.r_ok = ok; sh.r_small = so; }
    }
  }
  CT("phase1");
  // waves 0-2 meet without wave 3 (still doubling): an LDS counter, release / acquire
  if (lane == 0) __hip_atomic_fetch_add(&sh.ready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(&sh.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 3) __builtin_amdgcn_s_sleep(1);
  const int W = sh.W;
  if (wave == 2) {
    if (leaf) {
      fe ax, ay;
      _Pragma("unroll") for (int q = 0; q < 10; ++q) { ax.v[q] = sh.ax[q]; ay.v[q] = sh.ay[q]; }
      // [l - 2^252] A, l - 2^252 < 2^125: signed radix-16 digits (32 windows) over A's own table
      cold_table(sh.tab[2], gs_from_affine(ax, ay));
      const u32 delta[5] = {SC_L[0], SC_L[1], SC_L[2], SC_L[3], 0u};
      const Digits16 dg = recode16(delta, 32);
      i32 dv = dg.top;
      gs_p1p1 t = gs_cached_to_p1p1(cold_load(sh.tab[2][dv < 0 ? -dv : dv], dv < 0));
#pragma unroll 1
      for (int w = 30; w >= 0; --w) {
        gs_p2 p2 = gs_to_p2(t);
#pragma unroll 1
        for (int j = 0; j < 3; ++j) { t = gs_dbl(p2); p2 = gs_to_p2(t); }
        t = gs_dbl(p2);
        dv = digit16_of(dg, w, 32);
        t = gs_add_cached(gs_to_p3(t), cold_load(sh.tab[2][dv < 0 ? -dv : dv], dv < 0));
      }
      cold_store_p2(sh.dq, gs_to_p2(t));
      CT("deltaA");
    }
    __syncthreads();
    return;
  }
  if (wave == 0) {
    // the -d R terms: their own table and ladder (same windows and doublings as wave 1's)
    fe rx, ry;
    _Pragma("unroll") for (int q = 0; q < 10; ++q) { rx.v[q] = sh.rx[q]; ry.v[q] = sh.ry[q]; }
    cold_table(sh.tab[1], gs_from_affine(fe_neg(rx), ry));
    const Digits16 dd = sh.dd;
    i32 dr = dd.top;
    gs_p1p1 t = gs_cached_to_p1p1(cold_load(sh.tab[1][dr < 0 ? -dr : dr], dr < 0));
#pragma unroll 1
    for (int w = W - 2; w >= 0; --w) {
      gs_p2 p2 = gs_to_p2(t);
#pragma unroll 1
      for (int j = 0; j < 3; ++j) { t = gs_dbl(p2); p2 = gs_to_p2(t); }
      t = gs_dbl(p2);
      dr = digit16_of(dd, w, W);
      t = gs_add_cached(gs_to_p3(t), cold_load(sh.tab[1][dr < 0 ? -dr : dr], dr < 0));
    }
    cold_store(sh.rsum, gs_to_cached(gs_to_p3(t)));
    CT("Rshare");
    __syncthreads();
    return;
  }
  // wave 1: the -c A and s B terms
  fe ax, ay;
  _Pragma("unroll") for (int q = 0; q < 10; ++q) { ax.v[q] = sh.ax[q]; ay.v[q] = sh.ay[q]; }
  // -c A = |c| (c < 0 ? A : -A)
  cold_table(sh.tab[0], gs_from_affine(sh.c_neg ? ax : fe_neg(ax), ay));
  const Digits16 cd = sh.cd;
  i32 da = cd.top;
  gs_p1p1 t = gs_cached_to_p1p1(cold_load(sh.tab[0][da < 0 ? -da : da], da < 0));
#pragma unroll 1
  for (int w = W - 1; w >= 0; --w) {
    if (w != W - 1) {
      gs_p2 p2 = gs_to_p2(t);
#pragma unroll 1
      for (int j = 0; j < 3; ++j) { t = gs_dbl(p2); p2 = gs_to_p2(t); }
      t = gs_dbl(p2);
      da = digit16_of(cd, w, W);
      t = gs_add_cached(gs_to_p3(t), cold_load(sh.tab[0][da < 0 ? -da : da], da < 0));
    }
  }
  CT("Ashare");
  __syncthreads();   // wave 0's -d R share, wave 3's s B, waves 2 and 3's halves of the torsion test
  t = gs_add_cached(gs_to_p3(t), cold_load(sh.rsum, false));
  t = gs_add_cached(gs_to_p3(t), cold_load(sh.bsum, false));
  const bool ident = gs_is_identity(gs_to_p2(t));
  CT("final");
  bool torsion = false;
  if (leaf) {
    // u([l - 2^252] A) = (Z + Y : Z - Y);  same u  <=>  U (Z - Y) = W (Z + Y)
    fe U, Wm, Y, Z;
    _Pragma("unroll") for (int q = 0; q < 10; ++q) {
      U.v[q] = sh.tu[0][q]; Wm.v[q] = sh.tu[1][q]; Y.v[q] = sh.dq[1][q]; Z.v[q] = sh.dq[2][q];
    }
    const bool same = fe_is_zero(fe_sub(fe_mul(U, fe_sub(Z, Y)), fe_mul(Wm, fe_add(Z, Y))));
    torsion = sh.a_ok && !same;
  }
  if (lane == 0) {
    const bool strict = a.strict != 0;
    const bool ok = sh.s_ok && sh.a_ok && sh.r_ok && !(strict && (sh.a_small || sh.r_small));
    const bool fb = !torsion && (!sh.lat_ok || (a.force_fb_every && (i % a.force_fb_every) == 0));
    if (vbytes) {
      __hip_atomic_store(vbytes + i, (uint8_t)(0x80u | (!torsion && !fb && ok && ident ? 1u : 0u) | (fb ? 2u : 0u)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (torsion) {
      // randomized domain (a key with torsion): Err, whatever the equation says
    } else if (fb) {
      a.fb_list[atomicAdd(a.fb_count, 1u)] = (uint32_t)i;   // decided by k_verify_fallback
    } else if (ok && ident) {
      atomicOr(reinterpret_cast<unsigned long long*>(a.out_bits) + (i >> 6), 1ull << (i & 63));
    }
  }
}

__global__ __launch_bounds__(128) void k_verify_comb_wide(VerifyArgs a, CombArgs ca) {
  __shared__ fe sh_rx, sh_ry;
  __shared__ int sh_rok;
  const uint64_t i = blockIdx.x;
  if (i >= a.n) return;   // block-uniform
  const Committee& cm = a.committee;
  u32 mw[8], aw[8], sgw[16];
  load_inputs(a, i, mw, aw, sgw);
  const int lane = threadIdx.x & 63;
  u32 rw[8], sw[8];
  _Pragma("unroll") for (int q = 0; q < 8; ++q) { rw[q] = sgw[q]; sw[q] = sgw[8 + q]; }
  ge_p3 sum;
  int key = -1, kk = 0;   // wave 0 only: wave 1 (the critical path) starts on R at once
  if (threadIdx.x >= 64) {
    // wave 1: R (dalek decompression), its small-order flag.  The decompression -- this kernel's
    // critical path -- runs limb-sliced (fe_sliced.h: one element per 16-lane row, 1.8x shorter
    // dependent chain); every row computes the same element.
    fe X, Y;
    u32 yc[8];
    bool ok;
    decompress_sliced(rw, X, Y, yc, ok);
    if (lane == 0) {
      sh_rx = X;
      sh_ry = Y;
      sh_rok = ok && !(a.strict && ycanon_is_small_order(yc));
    }
  } else {
    // lanes 0..31: basepoint comb (radix 2^8) windows; lanes 32..32+W-1: key comb windows (W = 19)
    // windows; lanes 54..63 hold the identity
    key = committee_lookup(cm, aw);
    kk = key < 0 ? 0 : key;
    u32 kw[8], sd[8], kd[9];
    challenge(rw, aw, mw, kw);
    sc_recode_radix256(sw, sd);
    sc_recode_radix<KeyComb::bits, KeyComb::windows>(kw, kd);
    const bool bside = lane < 32;
    const int w = bside ? lane : min(lane - 32, KeyComb::windows - 1);
    const i32 d = bside ? digit256_at(sd, w) : digit_at<KeyComb::bits>(kd, w);
    ge_niels e = bside ? comb_load(ca.comb_base, BaseComb::entries, w, d)
                       : comb_load(cm.comb + (size_t)kk * COMB_PER_KEY, KeyComb::entries, w, d);
    if (lane >= 32 + KeyComb::windows) e = ge_niels_identity();
    sum = ge_p1p1_to_p3(ge_niels_to_p1p1(ge_niels_cneg(e, d < 0)));
#pragma unroll 1
    for (int m = 1; m < 64; m <<= 1) {
      const ge_p3 o = shfl_xor_p3(sum, m);
      sum = ge_p1p1_to_p3(ge_add_cached(sum, ge_p3_to_cached(o)));
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const u32 fl = cm.flags[kk];
    const bool flags_ok = key >= 0 && sc_lt_l(sw) && key_flags_ok(fl, a.strict != 0) && sh_rok;
    const bool eq = fe_is_zero(fe_sub(sum.X, fe_mul(sh_rx, sum.Z))) && fe_is_zero(fe_sub(sum.Y, fe_mul(sh_ry, sum.Z)));
    if (ca.vbytes) {
      // zero-copy latency launch: one byte per equation straight into pinned host memory; bit 7
      // marks it written, and the system-scope store goes out at once, so the host can return as
      // soon as every byte is in (no wait for the stream's completion signal)
      __hip_atomic_store(ca.vbytes + i, (uint8_t)(0x80u | (flags_ok && eq ? 1u : 0u) | (key < 0 ? 2u : 0u)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      if (key < 0) {
        if (ca.list) ca.list[atomicAdd(ca.count, 1u)] = ca.list_base + (uint32_t)i;
        else atomicOr(ca.count, 1u);   // latency launch: flag it, the host re-runs the general path
      }
      if (flags_ok && eq) atomicOr(reinterpret_cast<unsigned long long*>(a.out_bits) + (i >> 6), 1ull << (i & 63));
    }
  }
}

// ------------------------------------------------------------------------------- certificates
// cert c owns votes [voffs[c], voffs[c+1]); cert_ok bit c = AND of its leaf bits (empty -> 1);
// bad_bits = NOT leaf bits over valid vote indices.
__global__ void k_cert_reduce(const uint64_t* __restrict__ leaf_bits, const uint32_t* __restrict__ voffs,
                              uint64_t m, uint64_t nvotes, uint64_t* __restrict__ cert_bits,
                              uint64_t* __restrict__ bad_bits) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool ok = true;
  if (c < m) {
    const uint32_t a = voffs[c], b = voffs[c + 1];
    for (uint32_t v = a; v < b; ++v) ok = ok && ((leaf_bits[v >> 6] >> (v & 63)) & 1);
  }
  const uint64_t ballot = __ballot(ok && c < m);
  if ((threadIdx.x & 63) == 0 && c < m) cert_bits[c >> 6] = ballot;
  // bad bits: one word per thread
  const uint64_t words = (nvotes + 63) / 64;
  if (bad_bits && c < words) {
    uint64_t wv = ~leaf_bits[c];
    const uint64_t lo = c * 64;
    if (lo + 64 > nvotes) wv &= (nvotes - lo >= 64) ? ~0ull : ((1ull << (nvotes - lo)) - 1);
    bad_bits[c] = wv;
  }
}

// vote -> certificate index of the votes [lo, hi) of a host call (nwc_verify_batch_many): offs holds
// the absolute vote offsets of certificates c0 .. c0 + ncert (ncert + 1 entries).  One wave per
// certificate, its lanes over the certificate's votes (coalesced stores).
__global__ void k_cert_index(const uint32_t* __restrict__ offs, uint32_t c0, uint32_t ncert, uint64_t lo, uint64_t hi,
                             uint32_t* __restrict__ idx) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < ncert; w += nw) {
    const uint64_t a = max((uint64_t)offs[w], lo), b = min((uint64_t)offs[w + 1], hi);
    for (uint64_t v = a + lane; v < b; v += 64) idx[v - lo] = c0 + (uint32_t)w;
  }
}

// ------------------------------------------------------------------------------- SHA-512 digests
// digest32 of message i = data[offsets[i] .. (ends ? ends[i] : offsets[i+1])).  One lane per
// message.  One compression site for every block kind (a fully unrolled compression is ~3.3k
// instructions; three inlined copies would not share the instruction cache): each block's 16
// words come from 8 dwordx4 loads when the block is whole and the message start is 16-byte
// aligned, otherwise from byte loads with the FIPS 180-4 padding (0x80, zeros, 128-bit big-endian
// bit length) built in place.  Lanes of different lengths stay converged on the compression.
struct ShaBlock { uint64_t w[16]; };
__device__ __noinline__ ShaBlock sha_block_bytes(const uint8_t* p, uint64_t len, uint64_t b) {
  // bytes [128 b, 128 b + 128) of the padded message
  ShaBlock r;
  uint64_t* w = r.w;
  const uint64_t base = b << 7;
  const uint64_t padded_blocks = (len + 17 + 127) >> 7;
  _Pragma("unroll") for (int j = 0; j < 16; ++j) {
    uint64_t x = 0;
    _Pragma("unroll") for (int k = 0; k < 8; ++k) {
      const uint64_t idx = base + 8 * j + k;
      const uint32_t byte = idx < len ? p[idx] : (idx == len ? 0x80u : 0u);
      x = (x << 8) | byte;
    }
    w[j] = x;
  }
  if (b + 1 == padded_blocks) { w[14] = len >> 61; w[15] = len << 3; }
  return r;
}

__global__ __launch_bounds__(256, 2) void k_sha512_digest32(const uint8_t* __restrict__ data,
                                                            const uint64_t* __restrict__ offsets,
                                                            const uint64_t* __restrict__ ends,
                                                            uint64_t n, uint8_t* __restrict__ out32) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t start = offsets[i];
  const uint64_t len = (ends ? ends[i] : offsets[i + 1]) - start;
  const uint8_t* p = data + start;
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint64_t fast = (start & 15) == 0 ? (len >> 7) : 0;   // whole, aligned blocks
  const uint64_t total = (len + 17 + 127) >> 7;                 // blocks incl. padding
  uint64_t st[8];
  sha512_init_state(st);
#pragma unroll 1
  for (uint64_t b = 0; b < total; ++b) {
    uint64_t w[16];
    if (__builtin_expect(b < fast, 1)) {
      uint4 v[8];
      _Pragma("unroll") for (int j = 0; j < 8; ++j) v[j] = q[8 * b + j];
      _Pragma("unroll") for (int j = 0; j < 8; ++j) {
        w[2 * j] = be64_from_le32(v[j].x, v[j].y);
        w[2 * j + 1] = be64_from_le32(v[j].z, v[j].w);
      }
    } else {
      const ShaBlock r = sha_block_bytes(p, len, b);
      _Pragma("unroll") for (int j = 0; j < 16; ++j) w[j] = r.w[j];
    }
    sha512_compress<true>(st, w);
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(out32 + 32 * i);
  _Pragma("unroll") for (int j = 0; j < 4; ++j) {
    o[2 * j] = __builtin_bswap32((u32)(st[j] >> 32));
    o[2 * j + 1] = __builtin_bswap32((u32)st[j]);
  }
}

// ---- McNaughton-scheduled digests (many long messages) ---------------------------------------
// k_sha512_digest32 gives each lane one whole message, so a launch of n messages occupies
// ceil(n / 64) waves and the busiest SIMD runs ceil(n / 64 / SIMDs) of them one after another:
// at config 4 (100,000 batches, 1,563 waves on 1,024 SIMDs) half the SIMDs run two waves while
// the rest idle through the second.  Here every SIMD gets exactly one wave (256-thread
// workgroups, one per CU: the LDS reservation below admits a single workgroup per CU), and wave
// g owns the messages [g n / G, (g+1) n / G).  Its messages, laid end to end as a tape of
// compression blocks (S blocks in all, the longest M), are cut into 64 lane segments of
// T = max(ceil(S / 64), M) blocks; McNaughton's wrap-around rule makes that cut a valid schedule:
// a message that crosses the boundary between lanes l and l+1 has its FIRST a blocks compressed by
// lane l+1 at times [0, a) and its remaining blocks by lane l at the END of lane l's segment,
// which starts no earlier than time a because the message is no longer than T.  Lane l+1 hands
// the chaining value over through LDS (same wave: the write precedes the read in program order).
// Every lane prefetches the next block it will compress (and the next message's bounds) one
// compression ahead, so a single wave per SIMD keeps its VALU busy.
constexpr uint32_t SHA_NONE = 0xffffffffu;
struct ShaSchedLds {
  uint64_t st[4][8][64];     // per wave, per state word, per lane: handed-over chaining values
  uint32_t chain[4][64];     // per wave, per lane: first message of the lane's segment
  uint32_t off[4][64];       //                      and the tape offset of the segment in it
  uint8_t reserve[84 * 1024 - 4 * 8 * 64 * 8 - 2 * 4 * 64 * 4];   // > 80 KiB: one workgroup per CU
};
__device__ __forceinline__ uint64_t sha_msg_len(const uint64_t* offsets, const uint64_t* ends, uint64_t i) {
  return (ends ? ends[i] : offsets[i + 1]) - offsets[i];
}
__device__ __forceinline__ uint64_t sha_blocks(uint64_t len) { return (len + 17 + 127) >> 7; }

__global__ __launch_bounds__(256, 1) void k_sha512_digest32_sched(const uint8_t* __restrict__ data,
                                                                  const uint64_t* __restrict__ offsets,
                                                                  const uint64_t* __restrict__ ends,
                                                                  uint64_t n, uint8_t* __restrict__ out32) {
  __shared__ ShaSchedLds lds;
  const unsigned wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t G = (uint64_t)gridDim.x * 4, g = (uint64_t)blockIdx.x * 4 + wid;
  const uint64_t lo = g * n / G;
  const uint32_t cnt = (uint32_t)((g + 1) * n / G - lo);
  // tape length S and longest message M of this wave
  uint64_t S = 0, M = 0;
  for (uint32_t k = lane; k < cnt; k += 64) {
    const uint64_t L = sha_blocks(sha_msg_len(offsets, ends, lo + k));
    S += L;
    M = L > M ? L : M;
  }
  _Pragma("unroll") for (int d = 32; d >= 1; d >>= 1) {
    S += __shfl_xor(S, d);
    const uint64_t m2 = __shfl_xor(M, d);
    M = m2 > M ? m2 : M;
  }
  const uint64_t T = (S + 63) / 64 > M ? (S + 63) / 64 : M;
  // segment starts: message k covers tape [excl, incl); segment l starts at l T
  lds.chain[wid][lane] = SHA_NONE;
  lds.off[wid][lane] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  uint64_t carry = 0;
  for (uint32_t base = 0; base < cnt; base += 64) {
    const uint32_t k = base + lane;
    const uint64_t L = k < cnt ? sha_blocks(sha_msg_len(offsets, ends, lo + k)) : 0;
    uint64_t incl = L;
    _Pragma("unroll") for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(incl, d);
      if ((int)lane >= d) incl += y;
    }
    incl += carry;
    const uint64_t excl = incl - L;
    if (L) {
      const uint64_t l = (excl + T - 1) / T;
      if (l < 64 && l * T < incl) {
        lds.chain[wid][l] = k;
        lds.off[wid][l] = (uint32_t)(l * T - excl);
      }
    }
    carry = __shfl(incl, 63);
  }
  __syncthreads();

  uint32_t k = lds.chain[wid][lane];
  bool active = k != SHA_NONE;
  if (!active) k = 0;
  uint64_t c = lo + k;
  uint64_t start = 0, len = 0;
  if (active) { start = offsets[c]; len = sha_msg_len(offsets, ends, c); }
  uint64_t fast = (start & 15) == 0 ? (len >> 7) : 0;
  const uint32_t o = lds.off[wid][lane];
  uint64_t b = 0, e = sha_blocks(len) - o;   // first piece: the message's first blocks
  bool handoff = o != 0;                     // ... handed to lane - 1 when they end mid-message
  // bounds of the following message, one piece ahead
  uint64_t nstart = 0, nlen = 0;
  if (active && k + 1 < cnt) { nstart = offsets[c + 1]; nlen = sha_msg_len(offsets, ends, c + 1); }
  uint64_t st[8];
  sha512_init_state(st);
  uint4 v[8];
  if (active && b < fast) {
    const uint4* q = reinterpret_cast<const uint4*>(data + start);
    _Pragma("unroll") for (int j = 0; j < 8; ++j) v[j] = q[j];
  }
#pragma unroll 1
  for (uint64_t t = 0; t < T; ++t) {
    uint64_t w[16];
    if (active) {
      if (b < fast) {
        _Pragma("unroll") for (int j = 0; j < 8; ++j) {
          w[2 * j] = be64_from_le32(v[j].x, v[j].y);
          w[2 * j + 1] = be64_from_le32(v[j].z, v[j].w);
        }
      } else {
        const ShaBlock r = sha_block_bytes(data + start, len, b);
        _Pragma("unroll") for (int j = 0; j < 16; ++j) w[j] = r.w[j];
      }
    }
    // where this lane compresses next (index arithmetic only), and its prefetch
    const bool piece_end = active && b + 1 == e;
    bool nactive = active, fresh = false;
    uint64_t nb = b + 1, ne = e, pstart = start, plen = len;
    if (piece_end) {
      nactive = k + 1 < cnt && t + 1 < T;
      const uint64_t tot = sha_blocks(nlen), rem = T - (t + 1);
      fresh = tot <= rem;
      nb = fresh ? 0 : tot - rem;   // a message crossing into lane + 1: its last blocks only
      ne = tot;
      pstart = nstart;
      plen = nlen;
    }
    const uint64_t pfast = (pstart & 15) == 0 ? (plen >> 7) : 0;
    if (nactive && nb < pfast) {
      const uint4* q = reinterpret_cast<const uint4*>(data + pstart) + 8 * nb;
      _Pragma("unroll") for (int j = 0; j < 8; ++j) v[j] = q[j];
    }
    if (active) sha512_compress<true>(st, w);
    if (piece_end) {
      if (handoff) {
        _Pragma("unroll") for (int j = 0; j < 8; ++j) lds.st[wid][j][lane] = st[j];
      } else {
        uint32_t* op = reinterpret_cast<uint32_t*>(out32 + 32 * c);
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {
          op[2 * j] = __builtin_bswap32((u32)(st[j] >> 32));
          op[2 * j + 1] = __builtin_bswap32((u32)st[j]);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (nactive) {
        if (fresh) {
          sha512_init_state(st);
        } else {   // lane + 1 compressed this message's first nb blocks at times < t + 1
          _Pragma("unroll") for (int j = 0; j < 8; ++j) st[j] = lds.st[wid][j][lane + 1];
        }
        ++k;
        ++c;
        start = nstart;
        len = nlen;
        fast = pfast;
        if (k + 1 < cnt) { nstart = offsets[c + 1]; nlen = sha_msg_len(offsets, ends, c + 1); }
      }
      handoff = false;
    }
    active = nactive;
    b = nb;
    e = ne;
  }
}

// ------------------------------------------------------------------------------- keygen + sign
// Fixed-base scalar multiplication by a reduced scalar (< l) with the LDS base table.
__device__ __noinline__ ge_p3 base_scalarmult(const u32 a[8], const ge_niels* sB) {
  u32 sd[8];
  sc_recode_radix256(a, sd);
  ge_p3 acc = ge_p3_identity();
#pragma unroll 1
  for (int w = 31; w >= 0; --w) {
    if (w != 31) {
      ge_p2 p2 = ge_p3_to_p2(acc);
      ge_p1p1 t;
#pragma unroll 1
      for (int k = 0; k < 7; ++k) { t = ge_p2_dbl(p2); p2 = ge_p1p1_to_p2(t); }
      t = ge_p2_dbl(p2);
      acc = ge_p1p1_to_p3(t);
    }
    const i32 ds = (i32)(sd[7] >> 24) - 128;
    digits_shl(sd, 8);
    const int as = ds < 0 ? -ds : ds;
    acc = ge_p1p1_to_p3(ge_add_niels(acc, ge_niels_cneg(sB[as], ds < 0)));
  }
  return acc;
}

// Lane i: seed_i (32 B) and msg_i (32 B) -> pk_i (32 B), sig_i (64 B).  RFC 8032 / dalek:
//   h = SHA-512(seed); a = clamp(h[0..32]); A = aB; r = SHA-512(h[32..64] || M) mod l;
//   R = rB; k = SHA-512(R || A || M) mod l; s = r + k a mod l.
__global__ __launch_bounds__(256) void k_keygen_sign(const uint8_t* __restrict__ seeds,
                                                     const uint8_t* __restrict__ msgs, uint64_t n,
                                                     uint8_t* __restrict__ pks, uint8_t* __restrict__ sigs,
                                                     const ge_niels* __restrict__ base_table) {
  __shared__ ge_niels sB[129];
  for (int i = threadIdx.x; i < 129 * 30; i += blockDim.x)
    reinterpret_cast<i32*>(sB)[i] = reinterpret_cast<const i32*>(base_table)[i];
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u32 seed[8], m[8];
  load_words8(seeds + 32 * i, seed);
  load_words8(msgs + 32 * i, m);
  u32 sbuf[28];
  _Pragma("unroll") for (int j = 0; j < 28; ++j) sbuf[j] = j < 8 ? seed[j] : 0u;
  u32 h[16];
  sha512_one_block(sbuf, 32, h);
  u32 a[8];
  _Pragma("unroll") for (int j = 0; j < 8; ++j) a[j] = h[j];
  a[0] &= 0xFFFFFFF8u; a[7] &= 0x7FFFFFFFu; a[7] |= 0x40000000u;
  // a mod l (aB = (a mod l) B since B has order l)
  u32 wide[16];
  _Pragma("unroll") for (int j = 0; j < 16; ++j) wide[j] = j < 8 ? a[j] : 0u;
  u32 ar[8];
  sc_reduce512(wide, ar);
  u32 pk[8];
  ge_p3_compress(base_scalarmult(ar, sB), pk);
  u32 buf[28];
  _Pragma("unroll") for (int j = 0; j < 28; ++j) buf[j] = 0;
  _Pragma("unroll") for (int j = 0; j < 8; ++j) { buf[j] = h[8 + j]; buf[8 + j] = m[j]; }
  u32 rh[16];
  sha512_one_block(buf, 64, rh);
  u32 r[8];
  sc_reduce512(rh, r);
  u32 R[8];
  ge_p3_compress(base_scalarmult(r, sB), R);
  _Pragma("unroll") for (int j = 0; j < 8; ++j) { buf[j] = R[j]; buf[8 + j] = pk[j]; buf[16 + j] = m[j]; }
  u32 kh[16];
  sha512_one_block(buf, 96, kh);
  u32 k[8];
  sc_reduce512(kh, k);
  // s = (k * ar + r) mod l
  u32 prod[16];
  _Pragma("unroll") for (int j = 0; j < 16; ++j) prod[j] = 0;
  _Pragma("unroll") for (int x = 0; x < 8; ++x) {
    u64 carry = 0;
    _Pragma("unroll") for (int y = 0; y < 8; ++y) {
      u64 t = (u64)k[x] * ar[y] + prod[x + y] + carry;
      prod[x + y] = (u32)t;
      carry = t >> 32;
    }
    prod[x + 8] = (u32)carry;
  }
  u64 carry = 0;
  _Pragma("unroll") for (int j = 0; j < 16; ++j) {
    u64 t = (u64)prod[j] + (j < 8 ? r[j] : 0u) + carry;
    prod[j] = (u32)t;
    carry = t >> 32;
  }
  u32 s[8];
  sc_reduce512(prod, s);
  uint32_t* po = reinterpret_cast<uint32_t*>(pks + 32 * i);
  uint32_t* so = reinterpret_cast<uint32_t*>(sigs + 64 * i);
  _Pragma("unroll") for (int j = 0; j < 8; ++j) { po[j] = pk[j]; so[j] = R[j]; so[8 + j] = s[j]; }
}

}  // namespace nwc
#include "straus.h"
#include "msm.h"
#include "resolve.h"
namespace nwc {

// Seeds / messages of the synthetic workloads (SURVEY.md §8(d) cfg 2):
//   out_i = SHA-512(tag || u64le(first + i))[..32]
struct Tag64 { uint8_t b[64]; };
__global__ void k_derive32(Tag64 tag, int taglen, uint64_t first, uint64_t n, uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u32 words[28];
  _Pragma("unroll") for (int j = 0; j < 28; ++j) words[j] = 0;
  for (int b = 0; b < taglen; ++b) words[b >> 2] |= (u32)tag.b[b] << (8 * (b & 3));
  const uint64_t v = first + i;
  for (int b = 0; b < 8; ++b) {
    const int pos = taglen + b;
    words[pos >> 2] |= (u32)((v >> (8 * b)) & 0xFF) << (8 * (pos & 3));
  }
  u32 h[16];
  sha512_one_block(words, taglen + 8, h);
  uint32_t* o = reinterpret_cast<uint32_t*>(out + 32 * i);
  _Pragma("unroll") for (int j = 0; j < 8; ++j) o[j] = h[j];
}

}  // namespace nwc
