// dalek's verify_batch equation (ed25519-dalek 1.0.1 batch.rs, called by
// crypto/src/lib.rs:206-219 Signature::verify_batch) over sub-batches of votes, as a Straus
// multi-scalar multiplication per lane:
//
//     sum_i z_i R_i + sum_i (z_i k_i mod l) A_i - (sum_i z_i s_i mod l) B == O
//
// with random 128-bit z_i.  The votes of a launch (any certificates; each vote reads its own
// certificate digest) are cut into `runs` contiguous sub-batches of nq ~ 8-16 votes, one per lane
// at a time (persistent grid).  A lane runs Straus over its 2 nq points: the 63 x 4 doublings of
// its accumulator are shared by all of them, each window adds one entry per A_i (signed radix-16
// digits of z_i k_i mod l, 64 windows) and, in the low 33 windows, one per R_i (digits of z_i);
// then it adds -(sum z_i s_i mod l) B from the radix-2^22 basepoint comb (12 entries, no
// doublings) and tests the identity projectively.  No lane talks to another: a sub-batch that
// passes sets its votes' leaf bits, one that fails (a bad vote, an undecodable point, s >= l)
// lists its votes for the exact per-vote leaf kernel.  So at a bad-vote rate f only ~1-(1-f)^nq
// of the votes are verified twice, not every vote of a failing certificate.
//
// z_i = SHA-512(seed || u64le(global vote index))[..16], seed = 32 bytes the host draws per launch
// from its CSPRNG (dalek draws z_i from a merlin transcript finalised with thread_rng: both are
// 128-bit values the signers cannot predict).
//
// Semantics: on the deterministic domain (every vote ok, or some vote with
// a prime-order residual) the verdicts and the bad-vote set are exactly the leaves' (a sub-batch
// holding an err vote passes w.p. ~2^-125, as dalek's batch).  On dalek's randomized domain
// (pure-torsion residuals, torsion-bearing keys) a sub-batch passes w.p. ~1/ord, like dalek's
// batch -- where the leaf kernels answer Err deterministically -- so this is a separate entry
// point (nwc_dev_verify_batch_straus), not the default of nwc_verify_batch[_many].
#pragma once

namespace nwc {

#ifndef NWC_STRAUS_WAVES_PER_SIMD
#define NWC_STRAUS_WAVES_PER_SIMD 2
#endif
constexpr int STRAUS_WAVES_PER_SIMD = NWC_STRAUS_WAVES_PER_SIMD;
constexpr int STRAUS_MAX_PER_LANE = 16;
// per vote in a lane's scratch: A's and R's 9-entry tables, then the digit strings (64 B), padded
// to whole 128-B lines so every packed table entry of every vote is one cache line (an odd vote's
// entries straddled two lines with a 64-B digit block: 23 KB fetched per vote instead of ~13)
constexpr size_t STRAUS_VOTE_BYTES = (2 * TAB_BYTES_PER_LANE + 64 + 127) / 128 * 128;

struct StrausArgs {
  const uint8_t* digests;     // certificate digests, 32 B each
  const uint32_t* msg_index;  // per vote: its certificate (digest index)
  const uint8_t* pks;         // nv x 32
  const uint8_t* sigs;        // nv x 64
  uint64_t nv;
  uint64_t runs;              // sub-batch r = votes [r nv / runs, (r + 1) nv / runs), <= STRAUS_MAX_PER_LANE each
  uint32_t seed[8];
  const ge_niels_pad* comb16; // radix-2^22 basepoint comb
  uint8_t* scratch;           // lane_stride bytes per lane slot (lane-major: [lane slot][vote of run])
  uint64_t lane_stride;       // max votes per run * STRAUS_VOTE_BYTES
  uint64_t* leaf_words;       // bit v = vote v's sub-batch passed (zeroed by the caller)
  uint32_t* list;             // votes of the sub-batches that failed (for the exact leaves)
  uint32_t* count;
  // list mode (k_verify_straus<true>): the launch's votes are in_list[0 .. *in_count) (the votes of
  // the Pippenger groups that failed, msm.h), cut into runs on the device as straus_runs does;
  // lane_stride must then hold STRAUS_MAX_PER_LANE votes
  const uint32_t* in_list;
  const uint32_t* in_count;
  uint32_t target;
};

// 128-bit z of global vote index v
__device__ __forceinline__ void straus_z(const uint32_t seed[8], uint64_t v, u32 z[4]) {
  u32 words[28];
  _Pragma("unroll") for (int j = 0; j < 28; ++j) words[j] = 0;
  _Pragma("unroll") for (int j = 0; j < 8; ++j) words[j] = seed[j];
  words[8] = (u32)v;
  words[9] = (u32)(v >> 32);
  u32 h[16];
  sha512_one_block(words, 40, h);
  _Pragma("unroll") for (int j = 0; j < 4; ++j) z[j] = h[j];
}

// r = a * b mod l for a < 2^128 (4 words), b < 2^256 (8 words)
__device__ __forceinline__ void sc_mul128(const u32 a[4], const u32 b[8], u32 r[8]) {
  u32 prod[16];
  _Pragma("unroll") for (int i = 0; i < 16; ++i) prod[i] = 0;
  _Pragma("unroll") for (int x = 0; x < 4; ++x) {
    u64 carry = 0;
    _Pragma("unroll") for (int y = 0; y < 8; ++y) {
      const u64 t = (u64)a[x] * b[y] + prod[x + y] + carry;
      prod[x + y] = (u32)t;
      carry = t >> 32;
    }
    prod[x + 8] = (u32)carry;
  }
  sc_reduce512(prod, r);
}
// r = (a + b) mod l for a, b < l
__device__ __forceinline__ void sc_add_l(const u32 a[8], const u32 b[8], u32 r[8]) {
  u32 w[16];
  u64 c = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    const u64 t = (u64)a[i] + b[i] + c;
    w[i] = (u32)t;
    c = t >> 32;
  }
  w[8] = (u32)c;
  _Pragma("unroll") for (int i = 9; i < 16; ++i) w[i] = 0;
  sc_reduce512(w, r);
}

__device__ __forceinline__ ge_p3 shfl_xor_p3w(const ge_p3& p, int mask) {
  ge_p3 r;
  const fe* s = &p.X;
  fe* d = &r.X;
  _Pragma("unroll") for (int k = 0; k < 4; ++k)
    _Pragma("unroll") for (int i = 0; i < 10; ++i) d[k].v[i] = __shfl_xor(s[k].v[i], mask, 64);
  return r;
}

// digit w (0 = least significant) of a signed radix-16 nibble string (d + 8 per nibble)
__device__ __forceinline__ i32 nib_digit(const u32* words, int w) {
  return (i32)((words[w >> 3] >> (4 * (w & 7))) & 15u) - 8;
}

// Sub-batches of a launch of nv votes: each lane slot takes the same number of rounds, and the
// runs are as close to `target` votes as that allows (never more than STRAUS_MAX_PER_LANE).  A
// run costs ~253 doublings whatever it holds, so longer runs amortise them; a run with a bad vote
// is verified again vote by vote, so shorter runs re-verify less at a given bad-vote rate
// (target 12 by default, NWC_STRAUS_NQ to A/B).
__host__ __device__ inline uint64_t straus_runs(uint64_t nv, uint64_t lanes, uint32_t target) {
  if (target < 1) target = 1;
  if (target > (uint32_t)STRAUS_MAX_PER_LANE) target = STRAUS_MAX_PER_LANE;
  const uint64_t want = (nv + target - 1) / target;   // runs of <= target votes
  if (want <= lanes) return want;
  // every lane slot runs `rounds` sub-batches, of about `target` votes
  uint64_t rounds = (want + lanes / 2) / lanes;
  if (rounds < 1) rounds = 1;
  while ((nv + rounds * lanes - 1) / (rounds * lanes) > (uint64_t)STRAUS_MAX_PER_LANE) ++rounds;
  return rounds * lanes;
}

// The digit words of the current 8 windows, per vote of each lane, staged in LDS every 8 windows
// (row (2u + k) of 256 words, k = 0 the A digits, 1 the R digits; a wave's access is one 256-B row):
// the ladder's digit reads then never wait on memory in front of their table gathers.
constexpr int STRAUS_LDS_WORDS = 2 * STRAUS_MAX_PER_LANE * 256;

template <bool LIST = false>
__global__ __launch_bounds__(256, NWC_STRAUS_WAVES_PER_SIMD) void k_verify_straus(StrausArgs a) {
  __shared__ u32 dl[STRAUS_LDS_WORDS];
  const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  // vote t of lane slot l, lane-major ([l][t]; a vote-major layout measured no better,
  // profiles/r03/experiments.md)
  uint8_t* const base = a.scratch + slot * a.lane_stride;
  auto vote_base = [&](uint64_t t) { return base + t * STRAUS_VOTE_BYTES; };
  // entry 0 (the identity) of the first vote's tables: the add every lane of a wave makes in a
  // (window, vote) step where it has no vote of its own reads it
  LaneTable{reinterpret_cast<uint4*>(vote_base(0))}.store(0, ge_cached_identity());
  LaneTable{reinterpret_cast<uint4*>(vote_base(0) + TAB_BYTES_PER_LANE)}.store(0, ge_cached_identity());
  uint64_t nv = a.nv, runs = a.runs;
  if (LIST) {
    nv = *a.in_count;
    runs = straus_runs(nv, lanes, a.target);
  }
  // vote of position p: p itself, or in list mode the listed vote
  auto vote_at = [&](uint64_t p) -> uint64_t { return LIST ? (uint64_t)a.in_list[p] : p; };
  // persistent: lane slot l takes sub-batches l, l + lanes, ...
  for (uint64_t r0 = slot; ; r0 += lanes) {
    // wave-uniform loop exit: every lane of the wave leaves together
    const bool active = r0 < runs;
    if (!__any(active)) break;
    const uint64_t v0 = active ? r0 * nv / runs : 0, v1 = active ? (r0 + 1) * nv / runs : 0;
    const uint32_t nq = (uint32_t)(v1 - v0);
    bool ok = true;
    u32 S[8];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) S[i] = 0;
    // ---- phase 1: per vote, decode, scalars, tables
#pragma unroll 1
    for (uint32_t t = 0; t < nq; ++t) {
      const uint64_t v = vote_at(v0 + t);
      u32 mw[8], aw[8], sg[16];
      load_words8(a.digests + 32 * (uint64_t)a.msg_index[v], mw);
      load_words8(a.pks + 32 * v, aw);
      load_words8(a.sigs + 64 * v, sg);
      load_words8(a.sigs + 64 * v + 32, sg + 8);
      u32 kw[8], z[4], zk[8], zs[8];
      challenge(sg, aw, mw, kw);
      ok = ok && sc_lt_l(sg + 8);
      straus_z(a.seed, v, z);
      sc_mul128(z, kw, zk);
      sc_mul128(z, sg + 8, zs);
      sc_add_l(S, zs, S);
      uint8_t* vb = vote_base(t);
      // digit strings: z k mod l (64 signed radix-16 digits), z (33 digits of a < 2^128 value)
      u32* dg = reinterpret_cast<u32*>(vb + 2 * TAB_BYTES_PER_LANE);
      {
        u32 dk[8];
        sc_recode_radix16(zk, dk);
        u32 zz[8];
        _Pragma("unroll") for (int i = 0; i < 8; ++i) zz[i] = i < 4 ? z[i] : 0u;
        u32 dz[8];
        sc_recode_radix16(zz, dz);   // digits 33.. are zero (+8 nibbles)
        _Pragma("unroll") for (int i = 0; i < 8; ++i) { dg[i] = dk[i]; dg[8 + i] = dz[i]; }
      }
#pragma unroll 1
      for (int j = 0; j < 2; ++j) {
        u32 in[8];
        _Pragma("unroll") for (int i = 0; i < 8; ++i) in[i] = j ? sg[i] : aw[i];
        ge_p3 P;
        u32 yc[8];
        bool dok;
        ge_decompress1(in, P, yc, dok);
        ok = ok && dok;
        build_table(LaneTable{reinterpret_cast<uint4*>(vb + (size_t)j * TAB_BYTES_PER_LANE)}, P);
      }
    }
    // ---- phase 2: Straus over the lane's 2 nq points (shared doublings)
    ge_p1p1 t;
    t.X = fe_zero(); t.Y = fe_one(); t.Z = fe_one(); t.T = fe_one();   // identity (x = 0/1, y = 1/1)
    // every lane of the wave runs the same window/vote schedule: the wave's largest nq
    uint32_t nw = nq;
    _Pragma("unroll") for (int msk = 32; msk >= 1; msk >>= 1) nw = max(nw, (uint32_t)__shfl_xor((int)nw, msk, 64));
    nw = __builtin_amdgcn_readfirstlane(nw);
#pragma unroll 1
    for (int w = 63; w >= 0; --w) {
      if ((w & 7) == 7) {
        // stage the next 8 windows' digit words (a lane without vote u stages digit 0 = +8 nibbles)
#pragma unroll 1
        for (uint32_t u = 0; u < nw; ++u) {
          const u32* dg = reinterpret_cast<const u32*>(vote_base(u) + 2 * TAB_BYTES_PER_LANE);
          const bool has = u < nq;
          dl[(2 * u) * 256 + threadIdx.x] = has ? dg[w >> 3] : 0x88888888u;
          dl[(2 * u + 1) * 256 + threadIdx.x] = has ? dg[8 + (w >> 3)] : 0x88888888u;
        }
      }
      if (w != 63) ladder_dbl4(t);
      const int sh = 4 * (w & 7);
      // the window's additions in order A_0, R_0, A_1, R_1, ... (R only in the low 33 windows):
      // addition j = (vote j >> rs, kind j & rs); each one's first gather is issued an addition ahead
      const uint32_t rs = w <= 32 ? 1u : 0u, nadd = nw << rs;
      auto entry = [&](uint32_t j, i32& d, LaneTable& tab) {
        const uint32_t u = j >> rs, kind = j & rs;
        tab = LaneTable{reinterpret_cast<uint4*>(vote_base(u < nq ? u : 0) + kind * TAB_BYTES_PER_LANE)};
        d = (i32)((dl[(2 * u + kind) * 256 + threadIdx.x] >> sh) & 15u) - 8;
      };
      i32 dn;
      LaneTable tn;
      entry(0, dn, tn);
      uint4 qn[8];
      lt_load_full(tn, dn < 0 ? -dn : dn, dn < 0, qn);
#pragma unroll 1
      for (uint32_t j = 0; j < nadd; ++j) {
        const bool neg = dn < 0;
        uint4 cur[8];
        _Pragma("unroll") for (int k = 0; k < 8; ++k) cur[k] = qn[k];
        if (j + 1 < nadd) {
          entry(j + 1, dn, tn);
          lt_load_full(tn, dn < 0 ? -dn : dn, dn < 0, qn);
        }
        t = add_lt_full(t, cur, neg);
      }
    }
    // ---- phase 3: + (-S) B from the basepoint comb, identity test
    ge_p3 P = ge_p1p1_to_p3(t);
    // -S = l - S (S < l; S = 0 stays 0)
    u32 nS[8];
    {
      u64 br = 0;
      bool zero = true;
      _Pragma("unroll") for (int i = 0; i < 8; ++i) zero = zero && S[i] == 0;
      _Pragma("unroll") for (int i = 0; i < 8; ++i) {
        const u64 d = (u64)SC_L[i] - S[i] - br;
        nS[i] = zero ? 0u : (u32)d;
        br = (d >> 63) & 1;
      }
    }
    u32 sd[9];
    sc_recode_radix<NWC_BCOMB_BITS, COMB16_WINDOWS>(nS, sd);
#pragma unroll 1
    for (int w = COMB16_WINDOWS - 1; w >= 0; --w) {
      const i32 db = digit_at<NWC_BCOMB_BITS>(sd, w);
      const ge_niels e = comb_load(a.comb16, COMB16_ENTRIES, w, db);
      P = ge_p1p1_to_p3(ge_add_niels(P, ge_niels_cneg(e, db < 0)));
    }
    const bool ident = fe_is_zero(P.X) && fe_is_zero(fe_sub(P.Y, P.Z));
    if (active && nq) {
      if (ok && ident && LIST) {
        for (uint64_t p = v0; p < v1; ++p) {
          const uint64_t v = vote_at(p);
          atomicOr(reinterpret_cast<unsigned long long*>(a.leaf_words) + (v >> 6), 1ull << (v & 63));
        }
      } else if (ok && ident) {
        // the sub-batch's votes pass: set bits v0 .. v1-1 (at most two 64-bit words for nq <= 64)
        for (uint64_t wv = v0 >> 6; wv <= (v1 - 1) >> 6; ++wv) {
          const uint64_t lo = wv << 6;
          const uint32_t b0 = v0 > lo ? (uint32_t)(v0 - lo) : 0u;
          const uint32_t b1 = v1 - lo < 64 ? (uint32_t)(v1 - lo) : 64u;
          const uint64_t m = (b1 - b0 == 64 ? ~0ull : ((1ull << (b1 - b0)) - 1ull)) << b0;
          atomicOr(reinterpret_cast<unsigned long long*>(a.leaf_words) + wv, m);
        }
      } else {
        const uint32_t at = atomicAdd(a.count, nq);
        for (uint32_t q = 0; q < nq; ++q) a.list[at + q] = (uint32_t)vote_at(v0 + q);
      }
    }
  }
}


}  // namespace nwc
