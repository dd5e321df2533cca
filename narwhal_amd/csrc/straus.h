// dalek's verify_batch equation, per certificate, as a Straus multi-scalar multiplication
// (ed25519-dalek 1.0.1 batch.rs, called by crypto/src/lib.rs:206-219 Signature::verify_batch):
//
//     sum_i z_i R_i + sum_i (z_i k_i mod l) A_i - (sum_i z_i s_i mod l) B == O
//
// with random 128-bit z_i.  One certificate is split over L consecutive lanes of a wave (L chosen
// by the host, straus_lanes_per_cert, so that each lane holds at most STRAUS_MAX_PER_LANE votes
// and the persistent grid's last round is nearly full); lane q takes
// votes q, q + L, ... of its certificate and runs Straus over its 2 n_q points: the 63 x 4
// doublings of its accumulator are shared by all of them, each window adds one entry per A_i
// (signed radix-16 digits of z_i k_i mod l, 64 windows) and, in the low 33 windows, one per R_i
// (digits of z_i).  The L partial sums meet through lane shuffles; lane 0 of the group adds
// -(sum z_i s_i mod l) B from the radix-2^22 basepoint comb (12 entries, no doublings) and tests
// the identity projectively.
//
// z_i = SHA-512(seed || u64le(global vote index))[..16], seed = 32 bytes the host draws per launch
// from its CSPRNG (dalek draws z_i from a merlin transcript finalised with thread_rng: both are
// 128-bit values the signers cannot predict).
//
// Semantics: a vote that does not parse or decode (s >= l, A or R not on
// the curve) makes the certificate Err, as in dalek.  Otherwise this IS dalek's algorithm: Ok
// when every e_i = s_i B - k_i A_i - R_i is O and every A_i torsion-free; Err w.p. 1 - 2^-128-ish
// when some e_i has a prime-order component; and on dalek's randomized domain (pure-torsion
// residuals, torsion-bearing keys) Ok w.p. ~1/ord, like dalek -- where the leaf kernels answer Err
// deterministically.  A certificate that fails here is re-decided by the exact per-vote leaves
// (the bad-vote set), so only passing certificates' verdicts come from this kernel.
#pragma once

namespace nwc {

constexpr int STRAUS_MAX_PER_LANE = 24;
// per vote in a lane's scratch: A's and R's 9-entry tables, then the digit strings
constexpr size_t STRAUS_VOTE_BYTES = 2 * TAB_BYTES_PER_LANE + 64;

struct StrausArgs {
  const uint8_t* digests;     // m x 32 (one per certificate)
  const uint32_t* voffs;      // m + 1 vote offsets
  const uint8_t* pks;         // nv x 32
  const uint8_t* sigs;        // nv x 64
  uint64_t m;
  uint32_t lanes_per_cert;    // L: 1 .. 64
  uint32_t seed[8];
  const ge_niels_pad* comb16; // radix-2^22 basepoint comb
  uint8_t* scratch;           // lane_stride bytes per lane slot
  uint64_t lane_stride;       // ceil(max votes / L) * STRAUS_VOTE_BYTES
  uint64_t* cert_words;       // bit c = certificate c passed (zeroed by the caller)
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

// The digit words of the current 8 windows, per vote of each lane, staged in LDS every 8 windows
// (row (2u + k) of 256 words, k = 0 the A digits, 1 the R digits; a wave's access is one 256-B row):
// the ladder's digit reads then never wait on memory in front of their table gathers.
constexpr int STRAUS_LDS_WORDS = 2 * STRAUS_MAX_PER_LANE * 256;

__global__ __launch_bounds__(256, 2) void k_verify_straus(StrausArgs a) {
  __shared__ u32 dl[STRAUS_LDS_WORDS];
  const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const u32 L = a.lanes_per_cert;
  // groups of L consecutive lanes inside a wave (64 / L groups; the last 64 mod L lanes idle)
  const u32 lane = threadIdx.x & 63;
  const u32 gpw = 64u / L;
  const u32 gi = lane / L;
  const u32 q = lane - gi * L;
  const bool in_group = gi < gpw;
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t groups = waves * gpw;
  uint8_t* const base = a.scratch + slot * a.lane_stride;
  // entry 0 (the identity) of the first vote's tables: the add every lane of a wave makes in a
  // (window, vote) step where it has no vote of its own reads it
  LaneTable{reinterpret_cast<uint4*>(base)}.store(0, ge_cached_identity());
  LaneTable{reinterpret_cast<uint4*>(base + TAB_BYTES_PER_LANE)}.store(0, ge_cached_identity());
  // persistent: group g takes certificates g, g + groups, ...
  for (uint64_t c0 = (slot >> 6) * gpw + gi; ; c0 += groups) {
    // wave-uniform loop exit: every lane of the wave leaves together
    const bool active = in_group && c0 < a.m;
    if (!__any(active)) break;
    const uint64_t c = active ? c0 : 0;
    const uint32_t o0 = active ? a.voffs[c] : 0, o1 = active ? a.voffs[c + 1] : 0;
    const uint32_t nq = o1 > o0 + q ? (o1 - o0 - q + L - 1) / L : 0;
    u32 mw[8];
    load_words8(a.digests + 32 * c, mw);
    bool ok = true;
    u32 S[8];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) S[i] = 0;
    // ---- phase 1: per vote, decode, scalars, tables
#pragma unroll 1
    for (uint32_t t = 0; t < nq; ++t) {
      const uint64_t v = (uint64_t)o0 + q + (uint64_t)t * L;
      u32 aw[8], sg[16];
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
      uint8_t* vb = base + (size_t)t * STRAUS_VOTE_BYTES;
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
#pragma unroll 1
    for (int w = 63; w >= 0; --w) {
      if ((w & 7) == 7) {
        // stage the next 8 windows' digit words (a lane without vote u stages digit 0 = +8 nibbles)
#pragma unroll 1
        for (uint32_t u = 0; u < nw; ++u) {
          const u32* dg = reinterpret_cast<const u32*>(base + (size_t)u * STRAUS_VOTE_BYTES + 2 * TAB_BYTES_PER_LANE);
          const bool has = u < nq;
          dl[(2 * u) * 256 + threadIdx.x] = has ? dg[w >> 3] : 0x88888888u;
          dl[(2 * u + 1) * 256 + threadIdx.x] = has ? dg[8 + (w >> 3)] : 0x88888888u;
        }
      }
      if (w != 63) ladder_dbl4(t);
      const int sh = 4 * (w & 7);
      // the window's additions in order A_0, R_0, A_1, R_1, ... (R only in the low 33 windows):
      // addition j = (vote j / per, kind j % per); each one's first gather is issued an addition ahead
      const uint32_t per = w <= 32 ? 2u : 1u, nadd = nw * per;
      auto entry = [&](uint32_t j, i32& d, LaneTable& tab) {
        const uint32_t u = j / per, kind = j - u * per;
        tab = LaneTable{reinterpret_cast<uint4*>(base + (size_t)(u < nq ? u : 0) * STRAUS_VOTE_BYTES +
                                                 kind * TAB_BYTES_PER_LANE)};
        d = (i32)((dl[(2 * u + kind) * 256 + threadIdx.x] >> sh) & 15u) - 8;
      };
#if NWC_PACKED_TABLES
      i32 dn;
      LaneTable tn;
      entry(0, dn, tn);
      uint4 ab[4];
      lt_load_ab(tn, dn < 0 ? -dn : dn, dn < 0, ab);
#pragma unroll 1
      for (uint32_t j = 0; j < nadd; ++j) {
        const i32 d = dn;
        const LaneTable tab = tn;
        uint4 cur[4] = {ab[0], ab[1], ab[2], ab[3]};
        if (j + 1 < nadd) {
          entry(j + 1, dn, tn);
          lt_load_ab(tn, dn < 0 ? -dn : dn, dn < 0, ab);
        }
        t = add_lt_ab(t, cur, tab, d < 0 ? -d : d, d < 0);
      }
#else
#pragma unroll 1
      for (uint32_t j = 0; j < nadd; ++j) {
        i32 d;
        LaneTable tab;
        entry(j, d, tab);
        t = add_lt(t, tab, d < 0 ? -d : d, d < 0);
      }
#endif
    }
    // ---- phase 3: the group's partial sums (a segmented tree towards q = 0), -S B, identity test
    ge_p3 P = ge_p1p1_to_p3(t);
#pragma unroll 1
    for (u32 off = 1; off < L; off <<= 1) {
      ge_p3 Q;
      {
        const fe* sp = &P.X;
        fe* dp = &Q.X;
        _Pragma("unroll") for (int k = 0; k < 4; ++k)
          _Pragma("unroll") for (int i = 0; i < 10; ++i) dp[k].v[i] = __shfl_down(sp[k].v[i], off, 64);
      }
      u32 So[8];
      _Pragma("unroll") for (int i = 0; i < 8; ++i) So[i] = (u32)__shfl_down((int)S[i], off, 64);
      const bool oko = __shfl_down((int)ok, off, 64) != 0;
      if ((q & (2 * off - 1)) == 0 && q + off < L) {
        P = ge_p1p1_to_p3(ge_add_cached(P, ge_p3_to_cached(Q)));
        sc_add_l(S, So, S);
        ok = ok && oko;
      }
    }
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
    if (active && q == 0 && ok && ident)
      atomicOr(reinterpret_cast<unsigned long long*>(a.cert_words) + (c >> 6), 1ull << (c & 63));
  }
}

// Lanes per certificate for k_verify_straus: each lane pays ~252 doublings whatever it holds, and
// a persistent grid of G groups gives each group ceil(m / G) certificates in turn, so the
// last round can be nearly empty.  The host picks the L in 1..64 (any, not only powers of two)
// that minimises (per-vote work + the doublings' share) / (round efficiency x lanes used), with
// at most STRAUS_MAX_PER_LANE votes per lane.  Work in units of ~1k VALU instructions per vote.
inline uint32_t straus_lanes_per_cert(uint64_t m, uint32_t maxv, uint64_t resident_waves) {
  uint32_t best = 0;
  double best_cost = 1e300;
  for (uint32_t L = 1; L <= 64; ++L) {
    const uint32_t nq = (maxv + L - 1) / L;
    if (nq > (uint32_t)STRAUS_MAX_PER_LANE) continue;
    const uint32_t gpw = 64 / L;
    const double groups = (double)resident_waves * gpw;
    const double rounds = (double)m / groups;
    const double eff = (rounds / std::ceil(rounds)) * (double)(gpw * L) / 64.0;
    const double cost = (230.0 + 245.0 / (double)(nq ? nq : 1)) / eff;
    if (cost < best_cost) { best_cost = cost; best = L; }
  }
  return best;
}

// Largest certificate (votes) of a launch: one atomicMax per certificate (L is chosen from it).
__global__ void k_cert_maxlen(const uint32_t* __restrict__ voffs, uint64_t m, uint32_t* __restrict__ out) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < m) atomicMax(out, voffs[c + 1] - voffs[c]);
}

// After k_verify_straus: a vote of a passing certificate gets its leaf bit set; a vote of a failing
// one is listed for the exact leaf kernel (list mode ORs its verdict in), so that k_cert_reduce
// gives the certificate verdicts and the exact bad-vote set.  One wave per 64 votes.
__global__ void k_straus_expand(const uint64_t* __restrict__ cert_words, const uint32_t* __restrict__ msg_index,
                                uint64_t nv, uint64_t* __restrict__ leaf_words, uint32_t* __restrict__ list,
                                uint32_t* __restrict__ count) {
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = v < nv;
  const uint32_t c = in ? msg_index[v] : 0;
  const bool pass = in && ((cert_words[c >> 6] >> (c & 63)) & 1);
  const uint64_t bal = __ballot(pass);
  if ((threadIdx.x & 63) == 0 && v < nv) leaf_words[v >> 6] = bal;
  if (in && !pass) list[atomicAdd(count, 1u)] = (uint32_t)v;
}

}  // namespace nwc
