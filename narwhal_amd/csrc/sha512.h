// SHA-512 (FIPS 180-4) for gfx950, one message per lane.
//
// Used for (a) the worker batch digest `Sha512::digest(&batch)[..32]`
// (/root/reference/worker/src/processor.rs:38) and (b) the challenge H(R || A || M) inside
// verification (one 128-byte block: 96 message bytes + padding; messages are always the
// 32-byte `Digest` at the crypto surface, crypto/src/lib.rs:203,214).
//
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nwc {

__device__ __constant__ const uint64_t SHA512_K[80] = {
  0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL,0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL,0x12835b0145706fbeULL,0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL,0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,0x06ca6351e003826fULL,0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,0x53380d139d95b3dfULL,
  0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL,0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,
  0xca273eceea26619cULL,0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,0x113f9804bef90daeULL,0x1b710b35131c471bULL,
  0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL};

// 64-bit words live in VGPR pairs; every rotation is two v_alignbit_b32 on the halves, every
// three-input XOR / Ch / Maj one v_bitop3_b32 per half, every 64-bit add one v_lshl_add_u64
// (hipcc's own lowering of (x >> n) | (x << 64 - n) used 64-bit shifts plus ORs: ~5.1k VALU
// instructions per block against ~3.4k here).
__device__ __forceinline__ uint32_t sha_lo(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t sha_hi(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint64_t sha_pack(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }
// 64-bit add as one opaque v_lshl_add_u64: with a plain `+`, hipcc splits x + (hi << 32 | lo) into
// a zero-extended low add plus a high add, and moves the halves into pairs (~5 v_mov per round)
template <bool ASM> __device__ __forceinline__ uint64_t sha_add(uint64_t x, uint64_t y) {
  if constexpr (!ASM) return x + y;
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
// rotr(x, n) as (hi, lo) for a compile-time n in 1..63, n != 32
template <int N> __device__ __forceinline__ void sha_rotr2(uint64_t x, uint32_t& hi, uint32_t& lo) {
  static_assert(N > 0 && N < 64 && N != 32, "rotation");
  const uint32_t a = sha_hi(x), b = sha_lo(x);
  if constexpr (N < 32) {
    lo = __builtin_amdgcn_alignbit(a, b, N);
    hi = __builtin_amdgcn_alignbit(b, a, N);
  } else {
    lo = __builtin_amdgcn_alignbit(b, a, N - 32);
    hi = __builtin_amdgcn_alignbit(a, b, N - 32);
  }
}
// x >> n for 0 < n < 32
template <int N> __device__ __forceinline__ void sha_shr2(uint64_t x, uint32_t& hi, uint32_t& lo) {
  lo = __builtin_amdgcn_alignbit(sha_hi(x), sha_lo(x), N);
  hi = sha_hi(x) >> N;
}
constexpr unsigned SHA_XOR3 = 0x96, SHA_CH = 0xCA, SHA_MAJ = 0xE8;   // bitop3 truth tables (a, b, c)
#define NWC_SHA_BITOP3(a, b, c, OP)                                                                   \
  sha_pack(__builtin_amdgcn_bitop3_b32(sha_hi(a), sha_hi(b), sha_hi(c), OP),                          \
           __builtin_amdgcn_bitop3_b32(sha_lo(a), sha_lo(b), sha_lo(c), OP))
template <int A, int B, int C> __device__ __forceinline__ uint64_t sha_Sigma(uint64_t x) {
  uint32_t h0, l0, h1, l1, h2, l2;
  sha_rotr2<A>(x, h0, l0);
  sha_rotr2<B>(x, h1, l1);
  sha_rotr2<C>(x, h2, l2);
  return sha_pack(__builtin_amdgcn_bitop3_b32(h0, h1, h2, SHA_XOR3), __builtin_amdgcn_bitop3_b32(l0, l1, l2, SHA_XOR3));
}
template <int A, int B, int C> __device__ __forceinline__ uint64_t sha_sigma(uint64_t x) {
  uint32_t h0, l0, h1, l1, h2, l2;
  sha_rotr2<A>(x, h0, l0);
  sha_rotr2<B>(x, h1, l1);
  sha_shr2<C>(x, h2, l2);
  return sha_pack(__builtin_amdgcn_bitop3_b32(h0, h1, h2, SHA_XOR3), __builtin_amdgcn_bitop3_b32(l0, l1, l2, SHA_XOR3));
}

__device__ __forceinline__ void sha512_init_state(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL; st[2] = 0x3c6ef372fe94f82bULL;
  st[3] = 0xa54ff53a5f1d36f1ULL; st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
  st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// One compression: 5 passes of 16 statically unrolled rounds.  Round t of pass p uses schedule
// slot w[t & 15] = w[j] with j static, so the 16-word window stays in registers with no
// dynamic register indexing, and the a..h roles return to their places after 16 rounds (a
// multiple of 8).  Pass 0 (no message schedule) is peeled; passes 1-4 are one rolled loop.
//   Ch(e, f, g)  = (e & f) ^ (~e & g)          bitop3 0xCA
//   Maj(a, b, c) = (a & b) ^ (a & c) ^ (b & c) bitop3 0xE8
#define NWC_SHA_ROUND(a, b, c, d, e, f, g, h, J)                                                     \
  {                                                                                                  \
    if (SCHED) {                                                                                     \
      const uint64_t s0 = sha_sigma<1, 8, 7>(w[((J) + 1) & 15]);                                     \
      const uint64_t s1 = sha_sigma<19, 61, 6>(w[((J) + 14) & 15]);                                  \
      w[J] = sha_add<ASM>(sha_add<ASM>(w[J], s0), sha_add<ASM>(w[((J) + 9) & 15], s1));                             \
    }                                                                                                \
    const uint64_t S1 = sha_Sigma<14, 18, 41>(e);                                                    \
    const uint64_t ch = NWC_SHA_BITOP3(e, f, g, SHA_CH);                                             \
    const uint64_t t1 = sha_add<ASM>(sha_add<ASM>(h, k[J] + w[J]), sha_add<ASM>(S1, ch));                             \
    const uint64_t S0 = sha_Sigma<28, 34, 39>(a);                                                    \
    const uint64_t maj = NWC_SHA_BITOP3(a, b, c, SHA_MAJ);                                           \
    d = sha_add<ASM>(d, t1);                                                                              \
    h = sha_add<ASM>(t1, sha_add<ASM>(S0, maj));                                                               \
  }
#define NWC_SHA_16ROUNDS                                                                              \
  NWC_SHA_ROUND(a, b, c, d, e, f, g, h, 0)                                                           \
  NWC_SHA_ROUND(h, a, b, c, d, e, f, g, 1)                                                           \
  NWC_SHA_ROUND(g, h, a, b, c, d, e, f, 2)                                                           \
  NWC_SHA_ROUND(f, g, h, a, b, c, d, e, 3)                                                           \
  NWC_SHA_ROUND(e, f, g, h, a, b, c, d, 4)                                                           \
  NWC_SHA_ROUND(d, e, f, g, h, a, b, c, 5)                                                           \
  NWC_SHA_ROUND(c, d, e, f, g, h, a, b, 6)                                                           \
  NWC_SHA_ROUND(b, c, d, e, f, g, h, a, 7)                                                           \
  NWC_SHA_ROUND(a, b, c, d, e, f, g, h, 8)                                                           \
  NWC_SHA_ROUND(h, a, b, c, d, e, f, g, 9)                                                           \
  NWC_SHA_ROUND(g, h, a, b, c, d, e, f, 10)                                                          \
  NWC_SHA_ROUND(f, g, h, a, b, c, d, e, 11)                                                          \
  NWC_SHA_ROUND(e, f, g, h, a, b, c, d, 12)                                                          \
  NWC_SHA_ROUND(d, e, f, g, h, a, b, c, 13)                                                          \
  NWC_SHA_ROUND(c, d, e, f, g, h, a, b, 14)                                                          \
  NWC_SHA_ROUND(b, c, d, e, f, g, h, a, 15)
// ASM = true (the digest kernel): opaque 64-bit adds, -18 % instructions per block.  The verify
// kernels keep plain adds (ASM = false): their one challenge block is ~1 % of a verification,
// and the opaque adds cost them registers (more spills in the prologue).
// The digest kernels (ASM = true) run one wave per SIMD, where every scalar instruction takes an
// issue slot of its own: they fetch a pass's 16 round constants into SGPRs once per pass (two
// s_load_dwordx16 and one wait) instead of an address computation, a load and a wait per round.
template <bool ASM> __device__ __forceinline__ void sha_pass_constants(int pass, uint64_t k[16]) {
  _Pragma("unroll") for (int j = 0; j < 16; ++j) k[j] = SHA512_K[16 * pass + j];
  if constexpr (ASM) {
    _Pragma("unroll") for (int j = 0; j < 16; ++j) asm volatile("" : "+s"(k[j]));
  }
}
template <bool ASM = false> __device__ __forceinline__ void sha512_compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  {
    constexpr bool SCHED = false;   // rounds 0..15 use the message words as they are
    uint64_t k[16];
    sha_pass_constants<ASM>(0, k);
    NWC_SHA_16ROUNDS
  }
#pragma unroll 1
  for (int pass = 1; pass < 5; ++pass) {
    constexpr bool SCHED = true;
    uint64_t k[16];
    sha_pass_constants<ASM>(pass, k);
    NWC_SHA_16ROUNDS
  }
#undef NWC_SHA_16ROUNDS
#undef NWC_SHA_ROUND
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Big-endian 64-bit word from two little-endian-loaded 32-bit words (bytes b0..b7 in memory).
__device__ __forceinline__ uint64_t be64_from_le32(uint32_t lo, uint32_t hi) {
  return ((uint64_t)__builtin_bswap32(lo) << 32) | (uint64_t)__builtin_bswap32(hi);
}

}  // namespace nwc
