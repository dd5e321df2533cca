// dalek's verify_batch equation (ed25519-dalek 1.0.1 batch.rs, behind crypto/src/lib.rs:206-219)
// over groups of ~2-4k votes as a Pippenger multi-scalar multiplication with a wavefront-level
// bucket reduction (BASELINE.json north_star):
//
//     sum_i z_i R_i + sum_j (sum_{i: A_i = A_j} (z_i k_i mod l)) A_j - (sum_i z_i s_i mod l) B == O
//
// One wave owns a group of consecutive votes (any certificates; each vote reads its own
// certificate's digest), with random 128-bit z_i as in straus.h:
//
//   phase 1 (a vote per lane at a time): s < l, k_i = H(R||A||M) mod l, z_i, z_i k_i mod l and
//     z_i s_i mod l; R_i decompressed and stored in cached form (one 128-B line) with the
//     signed radix-2^10 digits of z_i; A_i's coefficient added into its key's accumulator in an LDS
//     hash table of the group's distinct keys (a committee's votes repeat ~100 keys: the A side
//     aggregates to one point per key, unreduced -- sum of the per-vote coefficients, < 2^265 --
//     so every vote keeps exactly dalek's coefficient); then one lane per distinct key decompresses
//     it and recodes its sum.
//   phase 2, Pippenger over the group's points, 14 windows of 10 bits from the top (z_i < 2^128
//     has digits in the low 13; a key's sum is split at 2^130 between A_j and 2^130 A_j): per
//     window the points are counting-sorted by |digit| into 512 buckets in LDS.  The window's
//     events in walking order -- for each bucket from the top, its points, then its end -- are
//     cut into 64 equal segments, lane l walking the l-th from the bottom: each point into a
//     running sum, at each bucket end the running sum into the lane's local total, so every lane
//     has the same number of events whatever the digits' distribution (a bucket may be shared by
//     two lanes).  The wavefront-level bucket reduction: sum_b b B_b = sum_l local_l +
//     sum_l beta_l SS_(l+1), where SS is the inclusive suffix scan of the lanes' running sums
//     (6 shuffle steps) and beta_l the bucket ends in lane l's segment (a short double-and-add);
//     each lane adds its term into its own Horner accumulator, and the 64 accumulators are summed
//     once, after the last window.
//   phase 3: - (sum z_i s_i mod l) B from the radix-2^22 basepoint comb, the identity test.
//
// A group that passes sets its votes' leaf bits; one that fails -- a vote that does not parse or
// decode, more than MSM_KMAX distinct keys, or the equation -- lists its votes for the exact
// per-vote leaves (list-mode k_verify), never for a second random equation.  Semantics (DESIGN.md
// §2.3, §4.2e): exact on the deterministic domain; on the randomized one a vote passes iff its
// group's equation holds.  The entry takes this path only when no key combs apply: otherwise it
// runs the comb leaves and dalek's equation per certificate (resolve.h).
#pragma once

namespace nwc {

constexpr int MSM_C = 10;                       // window bits
constexpr int MSM_BUCKETS = 1 << (MSM_C - 1);   // |digit| in 1 .. 512
constexpr int MSM_BW = MSM_BUCKETS / 64;        // buckets per lane in the counts' scan
constexpr int MSM_RWIN = 13;                    // windows of z < 2^128 (130 bits)
constexpr int MSM_WIN = 14;                     // windows of the group (a key's sum split at 2^130: < 2^135 each)
constexpr int MSM_KSPLIT = 130;                 // key point j: sum mod 2^130 on A_j, sum >> 130 on 2^130 A_j
constexpr int MSM_GMAX = 4096;                  // votes per group (at most)
constexpr int MSM_KMAX = 126;                   // distinct keys per group (at most; 126 keeps MsmLds in 1/8 of the LDS)
constexpr int MSM_SLOTS = 256;                  // LDS hash slots of the keys
constexpr u32 MSM_EMPTY = 0xFFFFFFFFu, MSM_CLAIMED = 0xFFFFFFFEu, MSM_FULL = 0xFFFFFFFDu;
constexpr int MSM_NPTS = MSM_GMAX + 2 * MSM_KMAX;   // R points, then A_j, then 2^130 A_j
constexpr size_t MSM_POINT_U4 = 8;              // one 128-B line per point: cached (Y+X, Y-X, Z, 2dT), packed
constexpr size_t MSM_WAVE_BYTES = (size_t)MSM_NPTS * MSM_POINT_U4 * 16 + (size_t)MSM_RWIN * MSM_GMAX * 2;

struct MsmArgs {
  const uint8_t* digests;     // certificate digests, 32 B each
  const uint32_t* msg_index;  // per vote: its certificate
  const uint8_t* pks;         // nv x 32
  const uint8_t* sigs;        // nv x 64
  uint64_t nv;
  uint32_t group;             // votes per group: a multiple of 64, <= MSM_GMAX
  uint32_t seed[8];
  const ge_niels_pad* comb16; // radix-2^22 basepoint comb
  uint8_t* scratch;           // MSM_WAVE_BYTES per block (one wave per block)
  uint64_t* leaf_words;       // bit v = vote v's group passed (zeroed by the caller)
  uint32_t* list;             // votes of the groups that failed (for the exact leaves)
  uint32_t* count;
  uint32_t* stats;            // MSM_ST_* words (nwc_msm_stats, the skip policy)
};

// device-resident MSM statistics and the skip policy's state (u32 words of DevCtx::msm_stats)
enum : int {
  MSM_ST_PASSED = 0,    // groups that passed the equation (cumulative)
  MSM_ST_FAILED = 1,    // groups that failed it (cumulative; a key overflow counts as failed)
  MSM_ST_OVERFLOW = 2,  // of them: more than MSM_KMAX distinct keys
  MSM_ST_MODE = 3,      // 0: the equation on every group; k = 1 .. MSM_SKIP_LAUNCHES - 1: on none (k-th such launch)
  MSM_ST_RUN = 4,       // this launch: groups the equation ran on
  MSM_ST_RUN_FAILED = 5,// this launch: of them, failed
  MSM_ST_SKIPPED = 6,   // groups handed to the leaves without the equation (cumulative)
  MSM_ST_WORDS = 8
};
// When more than half of a launch's groups fail (a bad-vote rate of ~1/group or more: every group
// holds one), the next MSM_SKIP_LAUNCHES - 1 launches skip the equation and pass every vote
// straight to the leaves (which a failing group's votes reach anyway, after a wasted MSM); the
// launch after them runs it on every group again to re-measure.  The state is per device (one
// set of words in DevCtx::msm_stats), shared by every caller and stream: one caller's bad launch
// makes the next launches of any caller skip the equation -- their verdicts are unchanged (the
// leaves are exact), only their speed (tests/test_gpu_msm.py).  Skipping within a
// launch would not help: a wave's group is latency-bound (one group alone takes as long as a full
// launch, profiles/r05/msm.md), so any probe costs a whole MSM launch -- 1 in 8 amortises it.
constexpr u32 MSM_SKIP_LAUNCHES = 8;

struct MsmLds {
  union {
    struct {
      u32 slots[MSM_SLOTS];
      u32 keys[MSM_KMAX][8];
      unsigned long long acc[MSM_KMAX][8];
      u32 nkeys, full;
    } p1;
    struct {
      u32 cnt[MSM_BUCKETS];
      u32 cur[MSM_BUCKETS];
      uint16_t sorted[MSM_NPTS];
    } p2;
  };
  int16_t kdig[2 * MSM_KMAX][MSM_WIN];   // the key points' digits (phase 1 end -> phase 2): A_j, then 2^130 A_j
};
// 8 waves per CU (2 per SIMD, the VGPR limit): a wave's group is latency-bound, so a CU holding 7
// (128 keys: 20,488 B) ran 1,775 larger groups in the time 2,048 smaller ones take
static_assert(sizeof(MsmLds) <= 160 * 1024 / 8, "MsmLds must leave room for 8 waves per CU");

// signed radix-2^10 digits (d in [-512, 511]) of a NWORDS-word number; the top window's value is
// small enough here (z < 2^128 in 13 windows, each half of a key sum < 2^135 in 14) that no carry
// leaves it
template <int NW, int NWORDS>
__device__ __forceinline__ void msm_recode(const u32 s[NWORDS], i32 out[NW]) {
  i32 carry = 0;
  _Pragma("unroll") for (int w = 0; w < NW; ++w) {
    const int b = MSM_C * w, wi = b >> 5, sh = b & 31;
    u32 v = wi < NWORDS ? s[wi] >> sh : 0u;
    if (sh > 32 - MSM_C && wi + 1 < NWORDS) v |= s[wi + 1] << (32 - sh);
    i32 d = (i32)(v & ((1u << MSM_C) - 1u)) + carry;
    carry = (d + (1 << (MSM_C - 1))) >> MSM_C;
    d -= carry << MSM_C;
    out[w] = d;
  }
}

__device__ __forceinline__ void msm_store_point(uint4* slot, const ge_p3& P) {
  // cached form, packed (a decompressed point has Z = 1; 2^130 A has not)
  const ge_cached q = ge_p3_to_cached(P);
  const fe c[4] = {q.YpX, q.YmX, q.Z, q.T2d};
  _Pragma("unroll") for (int k = 0; k < 4; ++k) {
    uint4 lo, hi;
    fe_pack(c[k], lo, hi);
    slot[2 * k] = lo;
    slot[2 * k + 1] = hi;
  }
}

__device__ __forceinline__ ge_p3 shfl_down_p3(const ge_p3& p, int delta) {
  ge_p3 r;
  const fe* s = &p.X;
  fe* d = &r.X;
  _Pragma("unroll") for (int k = 0; k < 4; ++k)
    _Pragma("unroll") for (int i = 0; i < 10; ++i) d[k].v[i] = __shfl_down(s[k].v[i], delta, 64);
  return r;
}
__device__ __forceinline__ ge_p3 p3_select(const ge_p3& a, const ge_p3& b, bool c) {
  ge_p3 r;
  r.X = fe_select(a.X, b.X, c);
  r.Y = fe_select(a.Y, b.Y, c);
  r.Z = fe_select(a.Z, b.Z, c);
  r.T = fe_select(a.T, b.T, c);
  return r;
}
__device__ __forceinline__ ge_p3 p3_add(const ge_p3& a, const ge_p3& b) {
  return ge_p1p1_to_p3(ge_add_cached(a, ge_p3_to_cached(b)));
}
__device__ __forceinline__ ge_p3 p3_dbl_n(ge_p3 p, int n) {
  ge_p2 q = ge_p3_to_p2(p);
  ge_p1p1 t;
#pragma unroll 1
  for (int i = 0; i < n - 1; ++i) {
    t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
  }
  t = ge_p2_dbl(q);
  return ge_p1p1_to_p3(t);
}

// The key of this lane's vote into the group's LDS key table (wave-uniform rounds, no spinning:
// a lane that finds an empty slot claims it with a CAS, the claimants publish their dense index
// after a barrier, and every pending lane then compares the 32 bytes of the slot's key).  Returns
// the dense index, -1 when the lane has no vote or the table is full (L.p1.full set).
__device__ int msm_key_index(MsmLds& L, const u32 aw[8], bool has) {
  u32 h = committee_hash(aw[0], aw[1]) & (MSM_SLOTS - 1);
  bool pending = has;
  int res = -1;
  u32 probes = 0;
  while (__any(pending)) {
    bool won = false;
    u32 k = MSM_FULL;
    if (pending && L.p1.slots[h] == MSM_EMPTY) won = atomicCAS(&L.p1.slots[h], MSM_EMPTY, MSM_CLAIMED) == MSM_EMPTY;
    if (won) {
      k = atomicAdd(&L.p1.nkeys, 1u);
      if (k < (u32)MSM_KMAX) {
        _Pragma("unroll") for (int i = 0; i < 8; ++i) L.p1.keys[k][i] = aw[i];
      } else {
        k = MSM_FULL;
      }
    }
    __syncthreads();
    if (won) L.p1.slots[h] = k;
    __syncthreads();
    if (pending) {
      const u32 s = L.p1.slots[h];
      if (s == MSM_FULL || ++probes > (u32)MSM_SLOTS) {
        L.p1.full = 1;
        pending = false;
      } else {
        u32 diff = 0;
        _Pragma("unroll") for (int i = 0; i < 8; ++i) diff |= L.p1.keys[s][i] ^ aw[i];
        if (diff == 0) {
          res = (int)s;
          pending = false;
        } else {
          h = (h + 1) & (MSM_SLOTS - 1);
        }
      }
    }
  }
  return res;
}

__global__ __launch_bounds__(64, 2) void k_verify_msm(MsmArgs a) {
  __shared__ MsmLds L;
  const u32 lane = threadIdx.x;
  uint8_t* const wbase = a.scratch + (size_t)blockIdx.x * MSM_WAVE_BYTES;
  uint4* const pts = reinterpret_cast<uint4*>(wbase);
  int16_t* const rdig = reinterpret_cast<int16_t*>(wbase + (size_t)MSM_NPTS * MSM_POINT_U4 * 16);
  const uint64_t G = a.group;
  const uint64_t ngroups = (a.nv + G - 1) / G;
  const bool skip = a.stats && a.stats[MSM_ST_MODE] != 0;
  for (uint64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint64_t v0 = g * G;
    const u32 ng = (u32)(a.nv - v0 < G ? a.nv - v0 : G);
    if (skip) {
      // skipped by the policy: the group's votes go to the Straus sub-batches as they are
      u32 at = 0;
      if (lane == 0) {
        at = atomicAdd(a.count, ng);
        atomicAdd(a.stats + MSM_ST_SKIPPED, 1u);
      }
      at = (u32)__shfl((int)at, 0, 64);
      for (u32 t = lane; t < ng; t += 64) a.list[at + t] = (uint32_t)(v0 + t);
      continue;
    }
    // ---------------- phase 1: scalars, R points, key aggregation
    for (u32 i = lane; i < (u32)MSM_SLOTS; i += 64) L.p1.slots[i] = MSM_EMPTY;
    for (u32 i = lane; i < (u32)MSM_KMAX * 8; i += 64) (&L.p1.acc[0][0])[i] = 0ull;
    if (lane == 0) {
      L.p1.nkeys = 0;
      L.p1.full = 0;
    }
    __syncthreads();
    bool ok = true;
    u32 S[8];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) S[i] = 0;
#pragma unroll 1
    for (u32 t0 = 0; t0 < ng; t0 += 64) {
      const u32 t = t0 + lane;
      const bool has = t < ng;
      const uint64_t v = v0 + (has ? t : 0);
      u32 mw[8], aw[8], sg[16];
      load_words8(a.digests + 32 * (uint64_t)a.msg_index[v], mw);
      load_words8(a.pks + 32 * v, aw);
      load_words8(a.sigs + 64 * v, sg);
      load_words8(a.sigs + 64 * v + 32, sg + 8);
      u32 kw[8], z[4], zk[8], zs[8];
      challenge(sg, aw, mw, kw);
      ok = ok && (!has || sc_lt_l(sg + 8));
      straus_z(a.seed, v, z);
      sc_mul128(z, kw, zk);
      sc_mul128(z, sg + 8, zs);
      if (has) sc_add_l(S, zs, S);
      ge_p3 R;
      u32 yc[8];
      bool dok;
      ge_decompress1(sg, R, yc, dok);
      ok = ok && (!has || dok);
      i32 dz[MSM_RWIN];
      msm_recode<MSM_RWIN, 4>(z, dz);
      if (has) {
        msm_store_point(pts + (size_t)t * MSM_POINT_U4, R);
        _Pragma("unroll") for (int w = 0; w < MSM_RWIN; ++w) rdig[(size_t)w * MSM_GMAX + t] = (int16_t)dz[w];
      }
      const int kidx = msm_key_index(L, aw, has);
      if (kidx >= 0)
        _Pragma("unroll") for (int i = 0; i < 8; ++i) atomicAdd(&L.p1.acc[kidx][i], (unsigned long long)zk[i]);
    }
    __syncthreads();
    const u32 K = min(L.p1.nkeys, (u32)MSM_KMAX);
    const bool full = L.p1.full != 0;
    // one lane per distinct key: its coefficient sum (exact, unreduced, < 2^265) split at 2^130 onto
    // A_j and 2^130 A_j (130 doublings), so the group's windows stop at 14 instead of 27
#pragma unroll 1
    for (u32 j0 = 0; j0 < K; j0 += 64) {
      const u32 j = j0 + lane;
      const bool has = j < K;
      const u32 jj = has ? j : 0;
      u32 sum[9];
      unsigned long long c = 0;
      _Pragma("unroll") for (int i = 0; i < 8; ++i) {
        const unsigned long long tsum = L.p1.acc[jj][i] + c;
        sum[i] = (u32)tsum;
        c = tsum >> 32;
      }
      sum[8] = (u32)c;
      // lo = sum mod 2^130, hi = sum >> 130 (< 2^135)
      u32 lo[5], hi[5];
      _Pragma("unroll") for (int i = 0; i < 4; ++i) {
        lo[i] = sum[i];
        hi[i] = (sum[4 + i] >> 2) | (sum[5 + i] << 30);
      }
      lo[4] = sum[4] & 3u;
      hi[4] = sum[8] >> 2;
      i32 dl[MSM_WIN], dh[MSM_WIN];
      msm_recode<MSM_WIN, 5>(lo, dl);
      msm_recode<MSM_WIN, 5>(hi, dh);
      u32 kw[8];
      _Pragma("unroll") for (int i = 0; i < 8; ++i) kw[i] = L.p1.keys[jj][i];
      ge_p3 A;
      u32 yc[8];
      bool dok;
      ge_decompress1(kw, A, yc, dok);
      ok = ok && (!has || dok);
      const ge_p3 A2 = p3_dbl_n(A, MSM_KSPLIT);
      if (has) {
        msm_store_point(pts + (size_t)(MSM_GMAX + j) * MSM_POINT_U4, A);
        msm_store_point(pts + (size_t)(MSM_GMAX + MSM_KMAX + j) * MSM_POINT_U4, A2);
        _Pragma("unroll") for (int w = 0; w < MSM_WIN; ++w) {
          L.kdig[j][w] = (int16_t)dl[w];
          L.kdig[MSM_KMAX + j][w] = (int16_t)dh[w];
        }
      }
    }
    // sum z_i s_i mod l over the wave
    _Pragma("unroll") for (int m = 32; m >= 1; m >>= 1) {
      u32 o[8];
      _Pragma("unroll") for (int i = 0; i < 8; ++i) o[i] = (u32)__shfl_xor((int)S[i], m, 64);
      sc_add_l(S, o, S);
    }
    const bool go = __all(ok) && !full;   // wave-uniform
    __syncthreads();                      // the phase-1 LDS (keys, accumulators) is dead from here
    bool pass = false;
    if (go) {
      // ---------------- phase 2: Pippenger windows from the top, per-lane Horner accumulators
      ge_p3 T = ge_p3_identity();
#pragma unroll 1
      for (int w = MSM_WIN - 1; w >= 0; --w) {
        if (w != MSM_WIN - 1) T = p3_dbl_n(T, MSM_C);
        // counting sort of the window's nonzero digits by |digit|
        for (u32 i = lane; i < (u32)MSM_BUCKETS; i += 64) L.p2.cnt[i] = 0;
        __syncthreads();
        const bool rwin = w < MSM_RWIN;
#pragma unroll 1
        for (u32 t = lane; rwin && t < ng; t += 64) {
          const i32 d = rdig[(size_t)w * MSM_GMAX + t];
          if (d) atomicAdd(&L.p2.cnt[(d < 0 ? -d : d) - 1], 1u);
        }
        for (u32 j = lane; j < 2 * K; j += 64) {
          const u32 kj = j < K ? j : MSM_KMAX + (j - K);
          const i32 d = L.kdig[kj][w];
          if (d) atomicAdd(&L.p2.cnt[(d < 0 ? -d : d) - 1], 1u);
        }
        __syncthreads();
        // exclusive scan of the counts (lane l scans buckets 8l .. 8l + 7): cnt[b] and cur[b]
        // become bucket b's start (the scatter below advances cur[b] to its end)
        u32 c8[MSM_BW], lsum = 0;
        _Pragma("unroll") for (int i = 0; i < MSM_BW; ++i) {
          c8[i] = L.p2.cnt[MSM_BW * lane + i];
          lsum += c8[i];
        }
        u32 incl = lsum;
        _Pragma("unroll") for (int o = 1; o < 64; o <<= 1) {
          const u32 y = (u32)__shfl_up((int)incl, o, 64);
          if ((int)lane >= o) incl += y;
        }
        const u32 npts = (u32)__shfl((int)incl, 63, 64);   // the window's points
        {
          u32 run = incl - lsum;
          _Pragma("unroll") for (int i = 0; i < MSM_BW; ++i) {
            L.p2.cnt[MSM_BW * lane + i] = run;
            L.p2.cur[MSM_BW * lane + i] = run;
            run += c8[i];
          }
        }
        __syncthreads();
#pragma unroll 1
        for (u32 t = lane; rwin && t < ng; t += 64) {
          const i32 d = rdig[(size_t)w * MSM_GMAX + t];
          if (d) {
            const u32 pos = atomicAdd(&L.p2.cur[(d < 0 ? -d : d) - 1], 1u);
            L.p2.sorted[pos] = (uint16_t)(t | (d < 0 ? 0x8000u : 0u));
          }
        }
        for (u32 j = lane; j < 2 * K; j += 64) {
          const u32 kj = j < K ? j : MSM_KMAX + (j - K);
          const i32 d = L.kdig[kj][w];
          if (d) {
            const u32 pos = atomicAdd(&L.p2.cur[(d < 0 ? -d : d) - 1], 1u);
            L.p2.sorted[pos] = (uint16_t)((MSM_GMAX + kj) | (d < 0 ? 0x8000u : 0u));
          }
        }
        __syncthreads();
        // The window's events in walking order D: for b = 511 .. 0, bucket b's points (from its
        // end down), then its end.  Lane l walks D[S_l, S_(l+1)) with S_l = (63 - l) * nte / 64:
        // every lane the same number of events whatever the digits' distribution (a lane may start
        // inside a bucket; a bucket may be shared by two lanes).  D index of bucket b's first event:
        // Dpos(b) = (npts - end(b)) + (511 - b), decreasing in b.
        const u32 nte = npts + (u32)MSM_BUCKETS;
        const u32 s_lo = (u32)(((uint64_t)(63 - lane) * nte) / 64), s_hi = (u32)(((uint64_t)(64 - lane) * nte) / 64);
        auto start_of = [&](int b) -> int { return (int)L.p2.cnt[b]; };   // bucket b's first sorted position
        auto end_of = [&](int b) -> int { return (int)L.p2.cur[b]; };     // one past its last
        auto dpos = [&](u32 b) -> u32 { return (npts - (u32)end_of((int)b)) + ((u32)MSM_BUCKETS - 1u - b); };
        u32 bfirst = 0;   // min b in [0, 511] with Dpos(b) <= s_lo (b = 511 always qualifies)
        {
          u32 lo = 0, hi = MSM_BUCKETS - 1;
          _Pragma("unroll") for (int it = 0; it < 9; ++it) {
            const u32 mid = (lo + hi) >> 1;
            const bool le = dpos(mid) <= s_lo;
            hi = (lo < hi && le) ? mid : hi;
            lo = (lo < hi && !le) ? mid + 1 : lo;
          }
          bfirst = lo;
        }
        const u32 nev = s_hi - s_lo;
        u32 E = nev;
        _Pragma("unroll") for (int m = 32; m >= 1; m >>= 1) E = max(E, (u32)__shfl_xor((int)E, m, 64));
        E = __builtin_amdgcn_readfirstlane(E);
        // the lane's events: each point into `run`, at a bucket's end `loc` += `run`
        ge_p3 run = ge_p3_identity(), loc = ge_p3_identity();
        int bi = (int)bfirst;
        int pos = end_of(bi) - 1 - (int)(s_lo - dpos(bfirst));   // below start(bi): the bucket's end
        // an event's kind and point depend only on (bi, pos), not on the additions: the next
        // event's 128-B point gather is issued before this event's arithmetic
        auto next_event = [&](u32 ev, bool& act, bool& is_pt, u32& id, uint4 (&pv)[MSM_POINT_U4]) {
          act = ev < nev;
          is_pt = act && bi >= 0 && pos >= start_of(max(bi, 0));
          id = is_pt ? (u32)L.p2.sorted[pos] : 0u;
          const uint4* e = pts + (size_t)(id & 0x7FFFu) * MSM_POINT_U4;
          _Pragma("unroll") for (int k = 0; k < (int)MSM_POINT_U4; ++k) pv[k] = e[k];
        };
        bool act_n, pt_n;
        u32 id_n;
        uint4 pn[MSM_POINT_U4];
        next_event(0, act_n, pt_n, id_n, pn);
#pragma unroll 1
        for (u32 ev = 0; ev < E; ++ev) {
          const bool act = act_n, is_pt = pt_n;
          const u32 id = id_n;
          uint4 pc[MSM_POINT_U4];
          _Pragma("unroll") for (int k = 0; k < (int)MSM_POINT_U4; ++k) pc[k] = pn[k];
          pos -= is_pt ? 1 : 0;
          bi -= (act && !is_pt) ? 1 : 0;
          if (ev + 1 < E) next_event(ev + 1, act_n, pt_n, id_n, pn);
          const bool neg = (id & 0x8000u) != 0;
          ge_cached q;
          {
            const fe ypx = fe_unpack(pc[0], pc[1]), ymx = fe_unpack(pc[2], pc[3]), pz = fe_unpack(pc[4], pc[5]),
                     t2d = fe_unpack(pc[6], pc[7]);
            const ge_cached qr = ge_p3_to_cached(run);
            q.YpX = fe_select(qr.YpX, neg ? ymx : ypx, is_pt);
            q.YmX = fe_select(qr.YmX, neg ? ypx : ymx, is_pt);
            q.Z = fe_select(qr.Z, pz, is_pt);
            q.T2d = fe_select(qr.T2d, neg ? fe_neg(t2d) : t2d, is_pt);
          }
          const ge_p3 tgt = p3_select(loc, run, is_pt);
          const ge_p3 r = ge_p1p1_to_p3(ge_add_cached(tgt, q));
          run = p3_select(run, r, is_pt);
          loc = p3_select(loc, r, act && !is_pt);
        }
        // Wavefront bucket reduction.  Every bucket end after lane l's segment counts its running
        // sum U_l once more: m_l = bi + 1 of them (the lane stopped before bucket bi's end), so the
        // window's sum_b (b + 1) B_b = sum_l loc_l + sum_l m_l U_l
        //                            = sum_l loc_l + sum_l beta_l SS_(l+1)   (Abel summation),
        // beta_l = m_(l+1) - m_l = the bucket ends in lane l's own segment (m_64 = 512) and
        // SS_(l+1) = sum_(k > l) U_k: an inclusive suffix scan of the running sums over the lanes
        // (6 shuffle steps), shifted by one lane, times beta_l (a short double-and-add: ~8, at most
        // 9 bits)
        ge_p3 ss = run;
        _Pragma("unroll 1") for (int o = 1; o < 64; o <<= 1) {
          const ge_p3 other = shfl_down_p3(ss, o);
          const ge_p3 sum = p3_add(ss, other);
          ss = p3_select(ss, sum, (int)lane + o < 64);
        }
        ss = p3_select(shfl_down_p3(ss, 1), ge_p3_identity(), lane == 63);   // SS_(l+1)
        const u32 m_l = (u32)(bi + 1);
        // (the shuffle outside the select: a shuffle inside a divergent branch reads the lanes
        // that skip it as 0)
        const u32 m_next = (u32)__shfl_down((int)m_l, 1, 64);
        const u32 m_up = lane == 63 ? (u32)MSM_BUCKETS : m_next;
        const u32 nb = m_up - m_l;
        u32 nbmax = nb;
        _Pragma("unroll") for (int m = 32; m >= 1; m >>= 1) nbmax = max(nbmax, (u32)__shfl_xor((int)nbmax, m, 64));
        const int bits = 32 - __builtin_clz(__builtin_amdgcn_readfirstlane(nbmax) | 1u);
        ge_p3 acc = ge_p3_identity();
#pragma unroll 1
        for (int k = bits - 1; k >= 0; --k) {
          acc = p3_dbl_n(acc, 1);
          acc = p3_select(acc, p3_add(acc, ss), ((nb >> k) & 1u) != 0);
        }
        T = p3_add(T, p3_add(loc, acc));
        __syncthreads();   // the window's LDS (counts, sorted) is rewritten by the next one
      }
      // the 64 lanes' accumulators
      _Pragma("unroll 1") for (int m = 32; m >= 1; m >>= 1) T = p3_add(T, shfl_xor_p3w(T, m));
      // - (sum z_i s_i mod l) B from the basepoint comb
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
        T = ge_p1p1_to_p3(ge_add_niels(T, ge_niels_cneg(e, db < 0)));
      }
      pass = fe_is_zero(T.X) && fe_is_zero(fe_sub(T.Y, T.Z));
      pass = __builtin_amdgcn_readfirstlane(pass ? 1 : 0) != 0;
    }
    if (pass) {
      // the group's votes pass: v0 is a multiple of 64, so its words are its own
      for (u32 k = lane; 64 * k < ng; k += 64) {
        const u32 nb = ng - 64 * k;
        const uint64_t m = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
        atomicOr(reinterpret_cast<unsigned long long*>(a.leaf_words) + (v0 >> 6) + k, m);
      }
    } else {
      u32 at = 0;
      if (lane == 0) at = atomicAdd(a.count, ng);
      at = (u32)__shfl((int)at, 0, 64);
      for (u32 t = lane; t < ng; t += 64) a.list[at + t] = (uint32_t)(v0 + t);
    }
    if (lane == 0 && a.stats) {
      atomicAdd(a.stats + (pass ? MSM_ST_PASSED : MSM_ST_FAILED), 1u);
      atomicAdd(a.stats + MSM_ST_RUN, 1u);
      if (!pass) atomicAdd(a.stats + MSM_ST_RUN_FAILED, 1u);
      if (full) atomicAdd(a.stats + MSM_ST_OVERFLOW, 1u);
    }
    __syncthreads();   // LDS of this group dead before the next group's phase 1
  }
}

// After each MSM launch (one thread): the next launch's mode (adapt = 0: the equation on every
// group).
__global__ void k_msm_policy(uint32_t* st, uint32_t adapt) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const u32 run = st[MSM_ST_RUN], failed = st[MSM_ST_RUN_FAILED];
  u32 mode = st[MSM_ST_MODE];
  if (!adapt) {
    mode = 0;
  } else if (mode != 0) {
    mode = mode + 1 < MSM_SKIP_LAUNCHES ? mode + 1 : 0;   // after the skipping launches, re-measure
  } else if (2 * failed > run) {
    mode = 1;
  }
  st[MSM_ST_MODE] = mode;
  st[MSM_ST_RUN] = 0;
  st[MSM_ST_RUN_FAILED] = 0;
}

}  // namespace nwc
