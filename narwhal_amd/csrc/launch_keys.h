// Launch keys: the committee a large batch-leaf launch brings with it (cross-certificate key
// aggregation).
//
// Certificate::verify (primary/src/messages.rs:189-215) only ever checks votes of committee members
// (a vote whose author has no stake is rejected before Signature::verify_batch, :203-214), so the
// 6.7M votes of BASELINE config 3 carry 100 distinct keys, each ~67k times.  A caller that never
// called nwc_set_committee still hands the library that repetition: a launch of >= LK_MIN_EQUATIONS
// batch-leaf equations samples LK_SAMPLES of its keys in one block (an LDS census), and every key
// seen at least LK_MIN_HITS times (a frequency of ~1/4096 or more) joins a device-resident key set
// -- its flags (decodes, small order, 8-torsion) and its radix-2^14 comb, built once -- after which
// the launch runs the committee comb kernel (k_verify_comb: 31 fixed-base additions per vote, no
// decompression) over it, and the votes of other keys take the per-vote ladder in list mode.  The
// set persists across launches (LK_MAX_KEYS keys; emptied by nwc_set_committee, by nwc_trim, and
// by a launch whose repeated keys it no longer covers -- see k_lk_select), so a node's steady
// state pays only the census.  Verdicts are those of the per-vote leaves: the key
// set changes which kernel decides a vote, never the verdict (tests/test_gpu_launch_keys.py).
//
// The whole pipeline stays on the launch's stream (no host synchronisation): k_lk_select (one
// block) updates the set, k_lk_keys / k_build_comb_from_bases build what joined (and exit at once otherwise), and
// k_verify_comb skips the comb sum of any wave none of whose equations has a held key.
#pragma once

namespace nwc {

constexpr u32 LK_MAX_KEYS = 128;       // keys held at most (20 MB of radix-2^14 comb each; allocated as keys join)
constexpr u32 LK_SLOTS = 1024;         // committee_lookup table of the held keys (load <= 1/8)
constexpr u32 LK_SAMPLES = 16384;      // equations sampled per launch
constexpr u32 LK_CENSUS = 8192;        // LDS census slots (power of two)
constexpr u32 LK_MIN_HITS = 4;         // sample hits that make a key join
constexpr int LK_PROBE = 32;
constexpr uint64_t LK_MIN_EQUATIONS = 65536;

struct LaunchKeys {
  u32* keys;            // LK_MAX_KEYS x 8 words
  u32* flags;           // KEY_DECODES | KEY_SMALL_ORDER | KEY_TORSION
  int32_t* slots;       // LK_SLOTS, -1 = empty
  ge_niels_pad* comb;   // cap x COMB_PER_KEY (grown by the host as keys ask to join)
  ge_p3* bases;         // LK_MAX_KEYS x KeyComb::windows
  u32* state;           // [0] keys held, [1] keys held before this launch's select, [2] keys it would hold
  u32* host_demand;     // host-mapped copy of state[2] (the host grows `comb` from it without a sync)
  u32 cap;              // keys `comb` has room for: joins stop there
};

__device__ __forceinline__ bool key_equal(const uint8_t* pks, u32 idx, const u32 aw[8]) {
  u32 kw[8];
  load_words8(pks + 32 * (uint64_t)idx, kw);
  u32 diff = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) diff |= kw[i] ^ aw[i];
  return diff == 0;
}

// One block of 1024 threads: LDS census of LK_SAMPLES equally spaced equations' keys, then the
// keys with >= LK_MIN_HITS hits that the set does not hold yet join it (in census-slot order).
// Replacement: when they do not all fit and the held keys cover less than a quarter of the
// sample's repeated-key hits (the node's committee changed -- an epoch change -- or the set filled
// with keys this traffic no longer carries), the set is emptied first and the launch's own
// repeated keys join it.  A set that still covers its share of the traffic keeps its keys, and
// the keys that do not fit take the per-vote ladder.
__global__ __launch_bounds__(1024) void k_lk_select(const uint8_t* pks, uint64_t n, LaunchKeys lk) {
  constexpr u32 EMPTY = 0xFFFFFFFFu;
  __shared__ u32 cidx[LK_CENSUS];
  __shared__ u32 ccnt[LK_CENSUS];
  __shared__ u32 fresh[LK_MAX_KEYS];
  __shared__ u32 nfresh, held_hits, fresh_hits, reset;
  for (u32 s = threadIdx.x; s < LK_CENSUS; s += blockDim.x) {
    cidx[s] = EMPTY;
    ccnt[s] = 0;
  }
  if (threadIdx.x == 0) {
    nfresh = 0;
    held_hits = 0;
    fresh_hits = 0;
    reset = 0;
  }
  __syncthreads();
  const uint64_t S = n < LK_SAMPLES ? n : LK_SAMPLES;
  for (uint64_t j = threadIdx.x; j < S; j += blockDim.x) {
    const u32 i = (u32)(j * n / S);
    u32 aw[8];
    load_words8(pks + 32 * (uint64_t)i, aw);
    const u32 h = committee_hash(aw[0], aw[1]);
    for (int p = 0; p < LK_PROBE; ++p) {
      const u32 slot = (h + p) & (LK_CENSUS - 1);
      const u32 old = atomicCAS(&cidx[slot], EMPTY, i);
      if (old == EMPTY || key_equal(pks, old, aw)) {
        atomicAdd(&ccnt[slot], 1u);
        break;
      }
    }
  }
  __syncthreads();
  const u32 held0 = lk.state[0];
  const Committee cur{lk.keys, lk.flags, nullptr, lk.comb, lk.slots, LK_SLOTS - 1, held0};
  for (u32 s = threadIdx.x; s < LK_CENSUS; s += blockDim.x) {
    if (cidx[s] == EMPTY || ccnt[s] < LK_MIN_HITS) continue;
    u32 aw[8];
    load_words8(pks + 32 * (uint64_t)cidx[s], aw);
    if (committee_lookup(cur, aw) >= 0) {
      atomicAdd(&held_hits, ccnt[s]);
      continue;
    }
    atomicAdd(&fresh_hits, ccnt[s]);
    const u32 k = atomicAdd(&nfresh, 1u);
    if (k < LK_MAX_KEYS) fresh[k] = cidx[s];
  }
  __syncthreads();
  if (threadIdx.x == 0) reset = (held0 + nfresh > LK_MAX_KEYS && 3u * held_hits < fresh_hits) ? 1u : 0u;
  __syncthreads();
  if (reset) {
    // every launch that read the set is ordered before this one (the caller's scratch_free wait)
    for (u32 s = threadIdx.x; s < LK_SLOTS; s += blockDim.x) lk.slots[s] = -1;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const u32 held = reset ? 0u : held0;
    // the keys that want to join and fit the policy's limit; those beyond the comb's allocated room
    // wait for the host to grow it (their votes take the ladder meanwhile)
    const u32 demand = min(held + nfresh, LK_MAX_KEYS);
    lk.state[2] = demand;
    if (lk.host_demand) *reinterpret_cast<volatile u32*>(lk.host_demand) = demand;
    const u32 add = min(nfresh, (lk.cap > held ? lk.cap : held) - held);
    u32 q = held;
    for (u32 k = 0; k < add; ++k) {
      u32 aw[8];
      load_words8(pks + 32 * (uint64_t)fresh[k], aw);
      const u32 h = committee_hash(aw[0], aw[1]);
      int p = 0;
      for (; p < COMMITTEE_MAX_PROBE; ++p) {
        int32_t* slot = &lk.slots[(h + p) & (LK_SLOTS - 1)];
        if (*slot < 0) {
          *slot = (int32_t)q;
          break;
        }
      }
      if (p == COMMITTEE_MAX_PROBE) continue;   // no free slot within the probe bound: not held
      _Pragma("unroll") for (int i = 0; i < 8; ++i) lk.keys[8 * q + i] = aw[i];
      ++q;
    }
    lk.state[1] = held;
    lk.state[0] = q;
  }
}

// One lane per key that joined: decode it, its flags (as k_build_key_tables: decodes, small
// order, l*A != O) and the comb's window bases 2^(14 w) (-A).
__global__ void k_lk_keys(LaunchKeys lk) {
  const u32 q = lk.state[1] + blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= lk.state[0]) return;
  u32 kw[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) kw[i] = lk.keys[8 * q + i];
  ge_p3 A;
  u32 yc[1][8];
  bool ok[1];
  const u32* const wp[1] = {kw};
  ge_decompressN<1>(&A, wp, yc, ok);
  lk.flags[q] = (ok[0] ? KEY_DECODES : 0u) | (ycanon_is_small_order(yc[0]) ? KEY_SMALL_ORDER : 0u) |
                (ok[0] && ge_has_torsion(A) ? KEY_TORSION : 0u);
  ge_p3 P = ge_p3_neg(A);
#pragma unroll 1
  for (int w = 0; w < KeyComb::windows; ++w) {
    lk.bases[(size_t)q * KeyComb::windows + w] = P;
#pragma unroll 1
    for (int k = 0; k < KeyComb::bits; ++k) P = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(P)));
  }
}

}  // namespace nwc
