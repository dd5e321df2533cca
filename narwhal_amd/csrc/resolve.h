// dalek's verify_batch equation decided per certificate from the exact per-vote leaves
// (crypto/src/lib.rs:206-219 -> ed25519-dalek 1.0.1 batch.rs).
//
// dalek accepts a certificate iff, for random 128-bit z_i,
//
//     -(sum z_i s_i mod l) B + sum z_i R_i + sum (z_i k_i mod l) A_i == O.
//
// With z_i k_i = (z_i k_i mod l) + q_i l and e_i = s_i B - R_i - k_i A_i the left side is
//     -sum_i (z_i e_i + q_i (l A_i)),
// and l A_i lies in the 8-torsion group E[8] (cyclic of order 8).  A vote whose leaf passed has
// e_i = O and l A_i = O: its term is O whatever z_i is.  So only the votes the leaves reject enter:
//   * a vote that does not parse or decode, or whose e_i has a prime-order component ([8] e_i != O),
//     makes the equation fail (with probability 1 - 2^-125: decided as Err);
//   * otherwise e_i and l A_i are in E[8] = <G8>: with e_i = [a_i] G8 and l A_i = [b_i] G8 the vote
//     contributes (z_i a_i + q_i b_i) mod 8, and the certificate passes iff its contributions sum
//     to 0 mod 8 -- dalek's own equation, evaluated exactly for these z_i, once per certificate.
// G8 = the order-8 point with y = SMALL_ORDER_Y[3] (encoding 26e8958f..6d53fc05, sign bit clear).
//
// k_vote_resolve takes the leaves' failing votes (list) one per lane: R' = s B - k A from the key's
// comb when the key is held (committee or launch keys: 31 fixed-base additions) or the full-length
// ladder otherwise, e = R' - R, [8] e; for the rare pure-torsion case also l A (a 252-doubling
// chain) and the two discrete logarithms.  Per certificate, cert_state = bit 31 "a vote failed
// deterministically" | the sum of contributions.  k_resolve_apply then sets the leaf bits of the
// listed votes of certificates whose state is 0 mod 8 with bit 31 clear (dalek's Ok), so
// cert_reduce reports them as passing; the other listed votes stay bad.
#pragma once

namespace nwc {

struct ResolveArgs {
  const uint8_t* digests;       // certificate digests, 32 B each
  const uint32_t* msg_index;    // per vote: its certificate (< m)
  const uint8_t* pks;           // nv x 32
  const uint8_t* sigs;          // nv x 64
  const uint32_t* list;         // the votes whose leaf failed
  const uint32_t* count;
  uint32_t seed[8];             // z_i = SHA-512(seed || u64le(i))[..16] (straus_z)
  Committee cm;                 // keys with combs (cm.comb == nullptr or n == 0: the ladder for every vote)
  const ge_niels_pad* comb16;   // radix-2^22 basepoint comb (comb_sum)
  const ge_niels* base_table;   // radix-256 basepoint table (the ladder)
  uint8_t* scratch;             // TAB_BYTES_PER_LANE per lane slot (the ladder's table of -A)
  uint32_t* cert_state;         // m words, zeroed by the caller
  uint64_t* leaf_words;         // k_resolve_apply: bit per vote
};

constexpr u32 RESOLVE_ERR = 0x80000000u;

// (X:Y:Z) == (X':Y':Z') projectively
__device__ __forceinline__ bool ge_p2_equal(const ge_p2& a, const ge_p2& b) {
  return fe_equal(fe_mul(a.X, b.Z), fe_mul(b.X, a.Z)) && fe_equal(fe_mul(a.Y, b.Z), fe_mul(b.Y, a.Z));
}

// l * P (double-and-add over l's bits, as ge_has_torsion)
__device__ __noinline__ ge_p2 ge_mul_l(const ge_p3& P) {
  const ge_cached pc = ge_p3_to_cached(P);
  ge_p2 acc = ge_p3_to_p2(P);   // bit 252
#pragma unroll 1
  for (int bit = 251; bit >= 0; --bit) {
    ge_p1p1 t = ge_p2_dbl(acc);
    if ((SC_L[bit >> 5] >> (bit & 31)) & 1u) t = ge_add_cached(ge_p1p1_to_p3(t), pc);
    acc = ge_p1p1_to_p2(t);
  }
  return acc;
}

// j in 0..7 with P == [j] G8 (P in E[8]); 8 if P is not in E[8]
__device__ __noinline__ u32 torsion_dlog(const ge_p2& P) {
  u32 gw[8];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) gw[i] = SMALL_ORDER_Y[3][i];
  ge_p3 G;
  u32 yc[8];
  bool ok;
  ge_decompress1(gw, G, yc, ok);
  const ge_cached gc = ge_p3_to_cached(G);
  ge_p3 acc = ge_p3_identity();
  u32 j = 8;
#pragma unroll 1
  for (u32 i = 0; i < 8; ++i) {
    if (j == 8 && ge_p2_equal(P, ge_p3_to_p2(acc))) j = i;
    acc = ge_p1p1_to_p3(ge_add_cached(acc, gc));
  }
  return j;
}

__global__ __launch_bounds__(256) void k_vote_resolve(ResolveArgs a) {
  __shared__ ge_niels sB[129];
  const uint32_t count = *a.count;
  if (count == 0) return;   // clean traffic: no failing vote, ~2 us
  stage_base_tables(a.base_table, sB, 129);
  const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const LaneTable tab{reinterpret_cast<uint4*>(a.scratch + slot * TAB_BYTES_PER_LANE)};
  const bool combs = a.cm.n != 0 && a.cm.comb != nullptr;
  const uint32_t stride = gridDim.x * blockDim.x;
  // wave-uniform trip count: every lane of a wave runs the same iterations (the comb and ladder
  // branches below are taken by the whole wave when any lane needs them)
  const uint32_t base0 = (uint32_t)slot & ~63u;
  for (uint32_t j0 = base0; j0 < count; j0 += stride) {
    const uint32_t j = j0 + (threadIdx.x & 63u);
    const bool active = j < count;
    const uint64_t v = active ? a.list[j] : a.list[0];
    u32 mw[8], aw[8], sgw[16];
    load_words8(a.digests + 32 * (uint64_t)a.msg_index[v], mw);
    load_words8(a.pks + 32 * v, aw);
    load_words8(a.sigs + 64 * v, sgw);
    load_words8(a.sigs + 64 * v + 32, sgw + 8);
    u32 rw[8], sw[8];
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { rw[i] = sgw[i]; sw[i] = sgw[8 + i]; }
    const bool s_ok = sc_lt_l(sw);
    u32 kw[8];
    challenge(rw, aw, mw, kw);
    const int key = combs ? committee_lookup(a.cm, aw) : -1;
    bool a_ok = key >= 0 && (a.cm.flags[key] & KEY_DECODES);
    ge_p2 rp;
    rp.X = fe_zero(); rp.Y = fe_one(); rp.Z = fe_one();
    if (__any(key >= 0)) {
      const ge_p2 q = comb_sum(sw, kw, a.comb16, a.cm.comb + (size_t)(key < 0 ? 0 : key) * COMB_PER_KEY);
      if (key >= 0) rp = q;
    }
    ge_p3 A;
    {
      u32 ya[8];
      bool ok;
      ge_decompress1(aw, A, ya, ok);
      if (key < 0) a_ok = ok;
    }
    if (__any(key < 0)) {
      build_table(tab, ge_p3_neg(A));
      u32 kd[8], sd[8];
      sc_recode_radix16(kw, kd);
      sc_recode_radix256(sw, sd);
      const ge_p2 q = double_scalarmult(tab, kd, sd, sB);
      if (key < 0) rp = q;
    }
    ge_p3 R;
    bool r_ok;
    {
      u32 yr[8];
      ge_decompress1(rw, R, yr, r_ok);
    }
    // e = R' - R: R' as an extended point (X Z : Y Z : Z^2 : X Y), plus -R
    ge_p3 rp3;
    rp3.X = fe_mul(rp.X, rp.Z); rp3.Y = fe_mul(rp.Y, rp.Z); rp3.Z = fe_sq(rp.Z); rp3.T = fe_mul(rp.X, rp.Y);
    const ge_p3 e = ge_p1p1_to_p3(ge_add_cached(rp3, ge_p3_to_cached(ge_p3_neg(R))));
    ge_p2 e8 = ge_p3_to_p2(e);
    _Pragma("unroll 1") for (int i = 0; i < 3; ++i) e8 = ge_p1p1_to_p2(ge_p2_dbl(e8));
    const bool torsion = fe_is_zero(e8.X) && fe_is_zero(fe_sub(e8.Y, e8.Z));
    const bool err = !(s_ok && a_ok && r_ok && torsion);
    u32 contrib = 0;
    bool dl_ok = true;
    if (active && !err) {
      // pure torsion residual: (z a + q b) mod 8 with e = [a] G8, l A = [b] G8 (rare: crafted votes)
      u32 z[4], zk[8];
      straus_z(a.seed, v, z);
      sc_mul128(z, kw, zk);
      const u32 z8 = z[0] & 7u, k8 = kw[0] & 7u, r8 = zk[0] & 7u;
      const u32 q8 = (5u * ((z8 * k8 + 8u - r8) & 7u)) & 7u;   // q = (z k - (z k mod l)) / l; 1/l = 5 mod 8
      const u32 de = torsion_dlog(ge_p3_to_p2(e));
      const u32 dl = torsion_dlog(ge_mul_l(A));
      dl_ok = de < 8 && dl < 8;
      contrib = (z8 * de + q8 * dl) & 7u;
    }
    if (active) {
      uint32_t* st = a.cert_state + a.msg_index[v];
      if (err || !dl_ok) atomicOr(st, RESOLVE_ERR);
      else if (contrib) atomicAdd(st, contrib);
    }
  }
}

// The listed votes of certificates dalek's equation accepts get their leaf bits.
__global__ __launch_bounds__(256) void k_resolve_apply(ResolveArgs a) {
  const uint32_t count = *a.count;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < count; j += gridDim.x * blockDim.x) {
    const uint32_t v = a.list[j];
    const u32 st = a.cert_state[a.msg_index[v]];
    if (!(st & RESOLVE_ERR) && (st & 7u) == 0)
      atomicOr(reinterpret_cast<unsigned long long*>(a.leaf_words) + (v >> 6), 1ull << (v & 63));
  }
}

// The votes [0, n) whose leaf bit is clear, appended to list / count (any order).
__global__ __launch_bounds__(256) void k_list_failing(const uint64_t* __restrict__ leaf_words, uint64_t n,
                                                     uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
  const uint64_t words = (n + 63) / 64;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t bad = ~leaf_words[w];
    if (w == words - 1 && (n & 63)) bad &= (1ull << (n & 63)) - 1;
    if (!bad) continue;
    uint32_t at = atomicAdd(count, (uint32_t)__popcll(bad));
    while (bad) {
      const int b = __ffsll((unsigned long long)bad) - 1;
      list[at++] = (uint32_t)(w * 64 + b);
      bad &= bad - 1;
    }
  }
}

}  // namespace nwc
