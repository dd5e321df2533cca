// Primary messages on the GPU: bincode/base64 ingestion, message digests and the structural
// checks of Header::verify / Vote::verify / Certificate::verify.
//
//   k_parse_messages     one wave per serialized PrimaryMessage (bincode 1.3 legacy config:
//                        little-endian fixint, u64 lengths; primary/src/primary.rs:230): the
//                        fixed fields are decoded by every lane alike, the certificate's votes
//                        one per lane (a vote is 116 B once its key string is 44 B, so vote v
//                        sits at a computed offset); decodes the base64 PublicKeys
//                        (crypto/src/lib.rs:94-112), gathers the Header::digest input
//                        (primary/src/messages.rs:70-84), computes Vote::digest (:145-153) and
//                        Certificate::digest (:226-234), evaluates the committee checks, and emits
//                        the signature equations: one strict equation per message (the header's
//                        or the vote's signature) and one batch-leaf equation per certificate vote.
//   k_header_digests     one lane per message: Header::digest of the gathered input vs the id.
//   k_finalize_messages  combines the flags with the equation verdicts into the DagError the
//                        reference returns, in its order (primary/src/error.rs).
//
// Wire layout (bincode of PrimaryMessage, primary/src/primary.rs:33-38):
//   u32 variant (0 Header, 1 Vote, 2 Certificate, 3 CertificatesRequest)
//   Header      = str author, u64 round, u64 P, P x (32-B digest, u32 worker id), u64 Q,
//                 Q x 32-B digest, 32-B id, 64-B signature
//   Vote        = 32-B id, u64 round, str origin, str author, 64-B signature
//   Certificate = Header, u64 V, V x (str key, 64-B signature)
//   str         = u64 length, bytes.
// Decoding follows the reference exactly:
//   * a PublicKey is a serde String decoded by PublicKey::decode_base64 (crypto/src/lib.rs:73-79):
//     base64 0.13 `decode` (b64_013_check below; padding optional, no trailing bits, '=' only at
//     the end of the last 8-symbol chunk) and `bytes[..32]`, which PANICS when fewer than 32 bytes
//     decode -- reported as DAG_DECODE_PANIC; longer decodes use their first 32 bytes.  Key strings
//     may have any length, so votes have no fixed stride (fast path: every key 44 bytes);
//   * Header.payload is a BTreeMap<Digest, WorkerId> and Header.parents a BTreeSet<Digest>
//     (primary/src/messages.rs:17-18): serde inserts the entries one by one, so the decoded header
//     -- and Header::digest (:75-81) and the worker check (:57-61) -- sees them sorted by digest
//     bytes, duplicates dropped, a map keeping the LAST value of a key (canon_set / canon_map);
//   * the first failing field in wire order decides between SerializationError and the panic;
//     trailing bytes after a message are ignored, as bincode's legacy config does.
#pragma once
#include <stdint.h>

namespace nwc {

enum DagCode : u32 {
  DAG_OK = 0,
  DAG_INVALID_SIGNATURE = 1,      // DagError::InvalidSignature
  DAG_INVALID_HEADER_ID = 2,      // DagError::InvalidHeaderId
  DAG_MALFORMED_HEADER = 3,       // DagError::MalformedHeader
  DAG_UNKNOWN_AUTHORITY = 4,      // DagError::UnknownAuthority
  DAG_AUTHORITY_REUSE = 5,        // DagError::AuthorityReuse
  DAG_REQUIRES_QUORUM = 6,        // DagError::CertificateRequiresQuorum
  DAG_TOO_OLD = 7,                // DagError::TooOld
  DAG_SERIALIZATION = 8,          // DagError::SerializationError
  DAG_UNEXPECTED_VOTE = 9,        // DagError::UnexpectedVote
  DAG_UNEXPECTED_MESSAGE = 10,    // CertificatesRequest (not a Core message)
  DAG_DECODE_PANIC = 11,          // the reference panics decoding a key (crypto/src/lib.rs:75 bytes[..32])
};
enum MsgKind : u32 { MSG_HEADER = 0, MSG_VOTE = 1, MSG_CERTIFICATE = 2, MSG_OTHER = 3 };

// Stake / worker tables of config::Committee (config/src/lib.rs:134-212), device resident.
struct CommitteeCfg {
  const uint64_t* stakes;      // per committee index (Committee::stake; 0 = no voting rights)
  const uint32_t* worker_off;  // n + 1
  const uint32_t* worker_ids;  // worker ids of authority k: [worker_off[k], worker_off[k+1])
  uint64_t quorum;             // 2 * total / 3 + 1 (Committee::quorum_threshold)
  uint32_t n;
};

// Core::sanitize_vote's expectation (the current header), optional
struct VoteTarget { u32 id[8]; u32 origin[8]; uint64_t round; int enabled; };

struct MsgArgs {
  const uint8_t* data;          // messages, 4-byte aligned base, >= 8 bytes of padding at the end
  const uint64_t* offsets;      // m + 1
  uint64_t m;
  uint64_t gc_round;            // Core::gc_round (TooOld for headers and certificates)
  VoteTarget target;
  uint8_t* hashbuf;             // per-message scratch for the header digest input
  // strict equations: one per message
  uint8_t* eq_msg;              // m x 32
  uint8_t* eq_pk;               // m x 32
  uint8_t* eq_sig;              // m x 64
  // batch-leaf equations: the certificates' votes
  uint8_t* v_pk;                // cap x 32
  uint8_t* v_sig;               // cap x 64
  uint32_t* v_msg;              // cap: equation -> message index (its certificate digest)
  uint8_t* cdig;                // m x 32: Certificate::digest per message (votes sign it)
  uint32_t* v_total;            // atomic vote-slot allocator
  uint64_t v_cap;
  uint32_t msg_base;            // the call-wide index of this launch's first message (v_msg entries)
  uint32_t* rec;                // m x 4: kind | flags << 8, post code, vote base, header digest input length
  uint32_t* rec_n;              // m: vote count
  uint32_t* hmatch;             // m: Header::digest == id (k_header_digests)
  uint8_t* digests;             // m x 32: the message's digest (Header::digest / Vote::digest /
                                //         Certificate::digest), for the caller
};

// ---- byte access: aligned dword loads + alignbyte (the data base is 4-byte aligned) --------
template <int K>
__device__ __forceinline__ void ld_words(const uint8_t* base, uint64_t off, u32 out[K]) {
  const u32* q = reinterpret_cast<const u32*>(base + (off & ~(uint64_t)3));
  const u32 sh = (u32)(off & 3);
  u32 w[K + 1];
  _Pragma("unroll") for (int i = 0; i <= K; ++i) w[i] = q[i];
  _Pragma("unroll") for (int i = 0; i < K; ++i) out[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}
__device__ __forceinline__ uint64_t ld_u64(const uint8_t* base, uint64_t off) {
  u32 w[2];
  ld_words<2>(base, off, w);
  return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
}
__device__ __forceinline__ u32 ld_u32(const uint8_t* base, uint64_t off) {
  u32 w[1];
  ld_words<1>(base, off, w);
  return w[0];
}

// standard base64 symbol value, or -1
__device__ __forceinline__ i32 b64_val(u32 c) {
  i32 v = -1;
  v = (c >= 'A' && c <= 'Z') ? (i32)c - 'A' : v;
  v = (c >= 'a' && c <= 'z') ? (i32)c - 'a' + 26 : v;
  v = (c >= '0' && c <= '9') ? (i32)c - '0' + 52 : v;
  v = (c == '+') ? 62 : v;
  v = (c == '/') ? 63 : v;
  return v;
}
// base64 0.13 `decode` (STANDARD config: standard alphabet, padding not required on decode,
// decode_allow_trailing_bits = false) of data[pos, pos + L), as PublicKey::decode_base64 runs it
// (crypto/src/lib.rs:73-79), followed by `bytes[..32]`:
//   KEY_ERR   a DecodeError: L % 8 in {1, 5}; a byte outside the alphabet ('=' included) in any
//             8-symbol chunk but the last; in the last chunk a '=' at a position i with i % 4 < 2
//             or a symbol after a '='; non-zero bits past the last whole output byte;
//   KEY_PANIC it decodes to fewer than 32 bytes (`bytes[..32]` panics);
//   KEY_OK    otherwise (the key is the first 32 decoded bytes = symbols 0..42, see b64_first32).
// Bytes >= 0x80 are never symbols, so the serde String's UTF-8 check cannot change the outcome.
// Restated in oracle/messages_ref.py b64_013_decode.
enum KeyStatus : u32 { KEY_OK = 0, KEY_ERR = 1, KEY_PANIC = 2 };
__device__ u32 b64_013_check(const uint8_t* base, uint64_t pos, uint64_t L) {
  if ((L & 3) == 1) return KEY_ERR;   // L % 8 in {1, 5}
  if (L == 0) return KEY_PANIC;       // decodes to nothing
  const uint64_t nch = (L + 7) >> 3;
  bool ok = true;
#pragma unroll 1
  for (uint64_t c = 0; c + 1 < nch; ++c) {
    u32 w[2];
    ld_words<2>(base, pos + 8 * c, w);
    _Pragma("unroll") for (int k = 0; k < 8; ++k) ok = ok && b64_val((w[k >> 2] >> (8 * (k & 3))) & 255u) >= 0;
  }
  const int tl = (int)(L - 8 * (nch - 1));
  u32 w[2];
  ld_words<2>(base, pos + 8 * (nch - 1), w);
  int k = 0;
  bool pad = false;
  uint64_t acc = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {
    if (i < tl) {
      const u32 c = (w[i >> 2] >> (8 * (i & 3))) & 255u;
      if (c == '=') {
        ok = ok && (i & 3) >= 2;
        pad = true;
      } else {
        const i32 v = b64_val(c);
        ok = ok && !pad && v >= 0;
        acc = (acc << 6) | (uint64_t)(v & 63);
        ++k;
      }
    }
  }
  // k is 2, 3, 4, 6, 7 or 8 here when ok (the length and padding rules exclude 0, 1 and 5)
  ok = ok && k >= 2 && k != 5;
  const int nb = (6 * k) >> 3, extra = 6 * k - 8 * nb;
  ok = ok && (acc & ((1ull << extra) - 1)) == 0;
  if (!ok) return KEY_ERR;
  return 6 * (nch - 1) + (uint64_t)nb < 32 ? KEY_PANIC : KEY_OK;
}
// The first 32 decoded bytes = the big-endian bits of symbols 0..42 (a decode of >= 32 bytes has
// >= 43 symbols, all before any padding): s[] holds characters 0..43 (character 43 is ignored).
__device__ __forceinline__ void b64_first32(const u32 s[11], u32 out[8]) {
  _Pragma("unroll") for (int i = 0; i < 8; ++i) out[i] = 0;
  _Pragma("unroll") for (int g = 0; g < 11; ++g) {
    u32 bits = 0;
    _Pragma("unroll") for (int k = 0; k < 4; ++k) {
      const i32 v = (4 * g + k < 43) ? b64_val((s[g] >> (8 * k)) & 255u) : 0;
      bits = (bits << 6) | (u32)(v & 63);
    }
    _Pragma("unroll") for (int b = 0; b < 3; ++b) {
      const int byte = 3 * g + b;
      if (byte < 32) out[byte >> 2] |= ((bits >> (16 - 8 * b)) & 255u) << (8 * (byte & 3));
    }
  }
}

// SHA-512[..32] of a 16-byte-aligned buffer (little-endian digest words)
__device__ void sha512_trunc32_buf(const uint8_t* p, uint64_t len, u32 out[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint64_t full = len >> 7;
  const uint64_t total = (len + 17 + 127) >> 7;
  uint64_t st[8];
  sha512_init_state(st);
#pragma unroll 1
  for (uint64_t b = 0; b < total; ++b) {
    uint64_t w[16];
    if (b < full) {
      _Pragma("unroll") for (int j = 0; j < 8; ++j) {
        const uint4 v = q[8 * b + j];
        w[2 * j] = be64_from_le32(v.x, v.y);
        w[2 * j + 1] = be64_from_le32(v.z, v.w);
      }
    } else {
      const ShaBlock r = sha_block_bytes(p, len, b);
      _Pragma("unroll") for (int j = 0; j < 16; ++j) w[j] = r.w[j];
    }
    sha512_compress(st, w);
  }
  _Pragma("unroll") for (int j = 0; j < 4; ++j) {
    out[2 * j] = __builtin_bswap32((u32)(st[j] >> 32));
    out[2 * j + 1] = __builtin_bswap32((u32)st[j]);
  }
}

// SHA-512[..32] of id(32) || round(8, LE) || key(32): Vote::digest, Certificate::digest
__device__ __forceinline__ void digest72(const u32 id[8], uint64_t round, const u32 key[8], u32 out[8]) {
  u32 wds[18];
  _Pragma("unroll") for (int i = 0; i < 8; ++i) { wds[i] = id[i]; wds[10 + i] = key[i]; }
  wds[8] = (u32)round;
  wds[9] = (u32)(round >> 32);
  u32 dg[16];
  sha512_one_block(wds, 72, dg);
  _Pragma("unroll") for (int i = 0; i < 8; ++i) out[i] = dg[i];
}

__device__ __forceinline__ void st_words(uint8_t* dst, const u32* w, int k) {
  u32* d = reinterpret_cast<u32*>(dst);
  for (int i = 0; i < k; ++i) d[i] = w[i];
}

struct MsgReader {
  const uint8_t* base;
  uint64_t pos, end;
  bool ok;
  bool panic;   // decoding stopped at a key whose base64 gives < 32 bytes (reference: panic)
  __device__ __forceinline__ bool need(uint64_t n) {
    ok = ok && pos <= end && n <= end - pos;
    return ok;
  }
  __device__ __forceinline__ uint64_t u64() {
    if (!need(8)) return 0;
    const uint64_t v = ld_u64(base, pos);
    pos += 8;
    return v;
  }
  __device__ __forceinline__ void bytes32(u32 out[8]) {
    if (!need(32)) { for (int i = 0; i < 8; ++i) out[i] = 0; return; }
    ld_words<8>(base, pos, out);
    pos += 32;
  }
  __device__ __forceinline__ void bytes64(u32 out[16]) {
    if (!need(64)) { for (int i = 0; i < 16; ++i) out[i] = 0; return; }
    ld_words<16>(base, pos, out);
    pos += 64;
  }
  // a PublicKey: serde String (u64 length, bytes) + PublicKey::decode_base64
  __device__ __forceinline__ void key(u32 out[8]) {
    for (int i = 0; i < 8; ++i) out[i] = 0;
    const uint64_t len = u64();
    if (!need(len)) return;
    const u32 st = b64_013_check(base, pos, len);
    if (st == KEY_OK) {
      u32 s[11];
      ld_words<11>(base, pos, s);   // < 44 bytes of string: the rest is padding / the next field
      b64_first32(s, out);
    } else {
      panic = st == KEY_PANIC;      // ok was true: this is the first failure
      ok = false;
    }
    pos += len;
  }
};

__device__ __forceinline__ bool words_eq8(const u32 a[8], const u32 b[8]) {
  u32 d = 0;
  _Pragma("unroll") for (int i = 0; i < 8; ++i) d |= a[i] ^ b[i];
  return d == 0;
}
__device__ __forceinline__ uint64_t member_stake(const CommitteeCfg& cc, int idx) {
  return idx >= 0 ? cc.stakes[idx] : 0;
}

// committees of up to this many authorities (the AuthorityReuse scan keeps one LDS slot each)
constexpr uint32_t MSG_MAX_COMMITTEE = 4096;
enum MsgFlag : u32 {
  MF_PARSE_ERR = 1u << 8,    // bincode / base64 decoding failed (or panicked, MF_PANIC)
  MF_GENESIS = 1u << 9,      // Certificate::genesis(committee).contains(self)
  MF_TOO_OLD = 1u << 10,     // gc_round > round (header, certificate)
  MF_STAKE0 = 1u << 11,      // the author has no voting rights
  MF_WORKER_BAD = 1u << 12,  // a payload worker id the author does not run
  MF_PANIC = 1u << 13,       // decoding reached a key of < 32 bytes before any error (panic)
};

__device__ __forceinline__ u32 wave_min_u32(u32 v) {
  _Pragma("unroll") for (int m = 32; m >= 1; m >>= 1) v = min(v, (u32)__shfl_xor((int)v, m, 64));
  return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  _Pragma("unroll") for (int m = 32; m >= 1; m >>= 1) {
    const u32 lo = (u32)__shfl_xor((int)(u32)v, m, 64), hi = (u32)__shfl_xor((int)(u32)(v >> 32), m, 64);
    v += (uint64_t)lo | ((uint64_t)hi << 32);
  }
  return v;
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  const u32 lo = (u32)__shfl((int)(u32)v, src, 64), hi = (u32)__shfl((int)(u32)(v >> 32), src, 64);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// ---- BTreeMap / BTreeSet from their bincode sequences (one wave) ----------------------------
// Digests order as byte strings (Digest derives Ord on [u8; 32]); the words are little-endian.
__device__ __forceinline__ int dig_cmp(const u32 a[8], const u32 b[8]) {
  int r = 0;
  _Pragma("unroll") for (int w = 7; w >= 0; --w) {
    const u32 x = __builtin_bswap32(a[w]), y = __builtin_bswap32(b[w]);
    r = x != y ? (x < y ? -1 : 1) : r;
  }
  return r;
}
// Writes the canonical form of `cnt` wire entries of WORDS words (digest first) at byte offset
// `src` into the word-aligned `dst` and returns the number of distinct digests:
//   SET (parents, 8 words): ascending digests, duplicates dropped (BTreeSet::insert keeps one);
//   MAP (payload, 9 words): ascending digests, one entry per digest with the LAST wire value
//        (serde's BTreeMap visitor inserts each entry; insert replaces an existing key's value).
// Strictly ascending input -- what serialising a BTree* produces -- is copied as is.  Otherwise
// the entries are sorted by (digest, wire index) -- up to CANON_RANK_MAX entries by rank (entry e
// goes to #smaller digests + #equal digests before it; cnt compares per entry), more by a bitonic
// network in dst (O(cnt log^2 cnt), so a Byzantine header of a maximum frame's worth of unsorted
// entries costs milliseconds, not the rank method's cnt^2 loads) -- and the sorted run is compacted
// in place 64 entries per step, keeping the first (SET) or the last (MAP) of each run of equal
// digests.  Every lane of the wave must call this.
constexpr uint64_t CANON_RANK_MAX = 512;

// (digest, tiebreak) order of two sort records; SET records tie-break on nothing (equal digests
// are equal records), MAP records carry the wire index in word 8 while they are sorted
template <bool MAP>
__device__ __forceinline__ bool canon_less(const u32 a[9], const u32 b[9]) {
  const int c = dig_cmp(a, b);
  return c < 0 || (MAP && c == 0 && a[8] < b[8]);
}

// Ascending sort of cnt records of W words in dst: the bitonic network whose comparators all put
// the minimum at the lower index (the first merge step of each block compares i with its mirror
// i ^ (k - 1)), so records past cnt act as +infinity and every comparator touching one is a no-op.
template <int W, bool MAP>
__device__ void canon_bitonic(u32* dst, uint64_t cnt, u32 lane) {
  uint64_t N = 1;
  while (N < cnt) N <<= 1;
  for (uint64_t k = 2; k <= N; k <<= 1) {
    for (uint64_t j = k >> 1; j >= 1; j >>= 1) {
      const bool flip = j == (k >> 1);
      for (uint64_t p = lane; p < N / 2; p += 64) {
        const uint64_t i = (p / j) * 2 * j + (p % j);
        const uint64_t l = flip ? (i ^ (k - 1)) : (i + j);
        if (l >= cnt) continue;
        u32 a[9], b[9];
        _Pragma("unroll") for (int w = 0; w < 9; ++w) {
          a[w] = w < W ? dst[W * i + w] : 0u;
          b[w] = w < W ? dst[W * l + w] : 0u;
        }
        if (canon_less<MAP>(b, a)) {
          _Pragma("unroll") for (int w = 0; w < W; ++w) {
            dst[W * i + w] = b[w];
            dst[W * l + w] = a[w];
          }
        }
      }
      __syncthreads();
    }
  }
}

template <int WORDS, bool MAP>
__device__ uint64_t canon_entries(const uint8_t* base, uint64_t src, uint64_t cnt, u32* dst, u32 lane) {
  constexpr uint64_t REC = 4 * WORDS;
  bool asc = true;
  for (uint64_t e = lane; e + 1 < cnt; e += 64) {
    u32 x[8], y[8];
    ld_words<8>(base, src + REC * e, x);
    ld_words<8>(base, src + REC * (e + 1), y);
    asc = asc && dig_cmp(x, y) < 0;
  }
  if (__all(asc)) {
    for (uint64_t k = lane; k < WORDS * cnt; k += 64) dst[k] = ld_u32(base, src + 4 * k);
    __syncthreads();
    return cnt;
  }
  if (cnt <= CANON_RANK_MAX) {
    for (uint64_t e = lane; e < cnt; e += 64) {
      u32 x[WORDS];
      ld_words<WORDS>(base, src + REC * e, x);
      uint64_t pos = 0;
#pragma unroll 1
      for (uint64_t j = 0; j < cnt; ++j) {
        u32 y[8];
        ld_words<8>(base, src + REC * j, y);
        const int c = dig_cmp(y, x);
        pos += (c < 0 || (c == 0 && j < e)) ? 1u : 0u;
      }
      _Pragma("unroll") for (int k = 0; k < WORDS; ++k) dst[WORDS * pos + k] = x[k];
    }
    __syncthreads();
  } else {
    // records (digest, wire index) for MAP, (digest) for SET, sorted in place; MAP's worker ids are
    // fetched back from the wire by index once the order is known
    for (uint64_t e = lane; e < cnt; e += 64) {
      u32 x[8];
      ld_words<8>(base, src + REC * e, x);
      _Pragma("unroll") for (int k = 0; k < 8; ++k) dst[WORDS * e + k] = x[k];
      if constexpr (MAP) dst[WORDS * e + 8] = (u32)e;
    }
    __syncthreads();
    canon_bitonic<WORDS, MAP>(dst, cnt, lane);
    if constexpr (MAP) {
      for (uint64_t e = lane; e < cnt; e += 64) dst[WORDS * e + 8] = ld_u32(base, src + REC * dst[WORDS * e + 8] + 32);
      __syncthreads();
    }
  }
  // Compaction: step s reads entries [64 s, 64 s + 64] and writes only below 64 s + 64, so no
  // step reads what an earlier step wrote; within a step every store depends on every load.
  uint64_t kept = 0;
  u32 carry[8];
  _Pragma("unroll") for (int k = 0; k < 8; ++k) carry[k] = 0;
  for (uint64_t t0 = 0; t0 < cnt; t0 += 64) {
    const uint64_t t = t0 + lane;
    const bool act = t < cnt;
    u32 x[WORDS];
    _Pragma("unroll") for (int k = 0; k < WORDS; ++k) x[k] = act ? dst[WORDS * t + k] : 0u;
    bool keep;
    if constexpr (MAP) {
      const bool last = t + 1 >= cnt;
      u32 y[8];
      _Pragma("unroll") for (int k = 0; k < 8; ++k) y[k] = (act && !last) ? dst[WORDS * (t + 1) + k] : 0u;
      keep = act && (last || dig_cmp(x, y) != 0);
    } else {
      u32 prev[8];
      _Pragma("unroll") for (int k = 0; k < 8; ++k) {
        prev[k] = (u32)__shfl_up((int)x[k], 1, 64);
        if (lane == 0) prev[k] = carry[k];
        carry[k] = (u32)__shfl((int)x[k], 63, 64);
      }
      keep = act && (t == 0 || dig_cmp(prev, x) != 0);
    }
    const uint64_t bal = __ballot(keep);
    const uint64_t at = kept + (uint64_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (keep) _Pragma("unroll") for (int k = 0; k < WORDS; ++k) dst[WORDS * at + k] = x[k];
    kept += (uint64_t)__popcll(bal);
  }
  __syncthreads();
  return kept;
}

// One wave (64-thread block) per message.  Every lane runs the sequential field decoding (same
// instructions, no divergence); vote-, payload- and digest-input loops are split across lanes.
// Dynamic LDS: one word per committee member (4 * min(cc.n, MSG_MAX_COMMITTEE) bytes, at least 4), so
// a 100-node committee takes 400 B per wave and the kernel's occupancy is set by its VGPRs.
__global__ __launch_bounds__(64) void k_parse_messages(MsgArgs a, Committee cm, CommitteeCfg cc) {
  extern __shared__ u32 first[];   // first vote position of each committee member
  const uint64_t i = blockIdx.x;
  const u32 lane = threadIdx.x;
  if (i >= a.m) return;   // block-uniform
  MsgReader r{a.data, a.offsets[i], a.offsets[i + 1], true, false};
  const uint64_t variant = ld_u32(a.data, r.pos);
  r.need(4);
  r.pos += 4;
  u32 kind = (r.ok && variant <= 2) ? (u32)variant : (u32)MSG_OTHER;
  u32 flags = 0, post = DAG_OK, vbase = 0, vcount = 0, hlen = 0;
  u32 eq_msg[8], eq_pk[8], eq_sig[16], dig[8], cd[8];
  _Pragma("unroll") for (int k = 0; k < 8; ++k) { eq_msg[k] = 0; eq_pk[k] = 0; dig[k] = 0; cd[k] = 0; }
  _Pragma("unroll") for (int k = 0; k < 16; ++k) eq_sig[k] = 0;
  if (kind == MSG_HEADER || kind == MSG_CERTIFICATE) {
    u32 author[8], id[8], sig[16];
    r.key(author);
    const uint64_t round = r.u64();
    const uint64_t P = r.u64();
    r.need(P <= (1ull << 40) ? P * 36 : ~0ull);
    const uint64_t pay_off = r.pos;
    if (r.ok) r.pos += P * 36;
    const uint64_t Q = r.u64();
    r.need(Q <= (1ull << 40) ? Q * 32 : ~0ull);
    const uint64_t par_off = r.pos;
    if (r.ok) r.pos += Q * 32;
    r.bytes32(id);
    r.bytes64(sig);
    const int aidx = r.ok ? committee_lookup(cm, author) : -1;
    const uint64_t astake = member_stake(cc, aidx);
    // per-message scratch (>= message length + 1 bytes, 128-B aligned): the Header::digest input
    // (author || round || BTreeMap payload || BTreeSet parents), then the vote offsets
    u32* d = reinterpret_cast<u32*>(a.hashbuf + ((a.offsets[i] + 127) & ~(uint64_t)127) + 128 * i);
    if (r.ok) {
      if (lane == 0) {
        _Pragma("unroll") for (int k = 0; k < 8; ++k) d[k] = author[k];
        d[8] = (u32)round;
        d[9] = (u32)(round >> 32);
      }
      const uint64_t Pc = canon_entries<9, true>(r.base, pay_off, P, d + 10, lane);
      const uint64_t Qc = canon_entries<8, false>(r.base, par_off, Q, d + 10 + 9 * Pc, lane);
      // Committee::worker(author, id) for every value of the map (only consulted for members)
      bool wbad = false;
      if (aidx >= 0) {
        const uint32_t w0 = cc.worker_off[aidx], w1 = cc.worker_off[aidx + 1];
        for (uint64_t e = lane; e < Pc; e += 64) {
          const u32 wid = d[10 + 9 * e + 8];
          bool found = false;
          for (uint32_t k = w0; k < w1; ++k) found = found || (cc.worker_ids[k] == wid);
          wbad = wbad || !found;
        }
      }
      if (__any(wbad)) flags |= MF_WORKER_BAD;
      hlen = (u32)(40 + 36 * Pc + 32 * Qc);
    }
    if (kind == MSG_CERTIFICATE) {
      const uint64_t V = r.u64();
      const uint64_t votes_off = r.pos;
      digest72(id, round, author, cd);
      // Vote positions.  Fast path: every key string is 44 bytes (base64::encode of 32 bytes), so
      // vote v sits at votes_off + 116 v -- true iff each of those length fields reads 44.
      bool fast = r.ok && V <= (r.end - r.pos) / 116;
      if (fast) {
        bool f = true;
        for (uint64_t v = lane; v < V; v += 64) f = f && ld_u64(r.base, votes_off + 116 * v) == 44;
        fast = __all(f);
      }
      // Otherwise lane 0 walks the list: voff[v] = offset of vote v for the nfull votes wholly
      // inside the message; `tail` = 1 when the next vote's key string is inside but its signature
      // is cut (its key still decides panic vs error), 2 when its length or key is cut.
      u32* voff = d + 12 + 9 * P + 8 * Q;   // past the digest input (P, Q >= the kept counts)
      uint64_t nfull = V;
      u32 tail = 0;
      if (r.ok && !fast) {
        uint64_t nf = 0;
        u32 tk = 0;
        if (lane == 0) {
          uint64_t cur = votes_off;
          for (; nf < V; ++nf) {   // every vote takes >= 72 bytes: ends within the message
            if (r.end - cur < 8) { tk = 2; break; }
            const uint64_t L = ld_u64(r.base, cur);
            if (L > r.end - cur - 8) { tk = 2; break; }
            voff[nf] = (u32)(cur - votes_off);
            if (r.end - cur - 8 - L < 64) { tk = 1; break; }
            cur += 8 + L + 64;
          }
        }
        nfull = shfl_u64(nf, 0);
        tail = (u32)__shfl((int)tk, 0, 64);
        __syncthreads();   // voff written by lane 0
      }
      const bool whole = r.ok && nfull == V;
      if (whole) {
        u32 vb = 0;
        if (lane == 0) vb = atomicAdd(a.v_total, (uint32_t)V);
        vbase = (u32)__shfl((int)vb, 0, 64);
        if ((uint64_t)vbase + V > a.v_cap) r.ok = false;   // cannot happen: v_cap >= bytes / 72
      }
      if (r.ok) {
        const uint32_t ncm = cc.n < MSG_MAX_COMMITTEE ? cc.n : MSG_MAX_COMMITTEE;
        for (uint32_t k = lane; k < ncm; k += 64) first[k] = 0xFFFFFFFFu;
        __syncthreads();
        // pass 1: decode every vote (one per lane).  The first failing vote in wire order decides
        // the message (bincode stops there); a whole list also emits its equations and notes
        // each member's first position.
        const uint64_t ndec = nfull + (tail == 1 ? 1 : 0);
        u32 fpos = 0xFFFFFFFFu, fkind = KEY_OK;
        uint64_t weight = 0;
        for (uint64_t v = lane; v < ndec; v += 64) {
          const uint64_t off = votes_off + (fast ? 116 * v : (uint64_t)voff[v]);
          MsgReader vr{a.data, off, r.end, true, false};
          u32 key[8], sg[16];
          vr.key(key);
          const u32 st = vr.ok ? (v < nfull ? KEY_OK : KEY_ERR) : (vr.panic ? KEY_PANIC : KEY_ERR);
          if (st != KEY_OK && (u32)v < fpos) { fpos = (u32)v; fkind = st; }
          if (!whole) continue;
          vr.bytes64(sg);
          st_words(a.v_pk + 32 * (vbase + v), key, 8);
          st_words(a.v_sig + 64 * (vbase + v), sg, 16);
          a.v_msg[vbase + v] = a.msg_base + (uint32_t)i;
          const int kidx = committee_lookup(cm, key);
          weight += member_stake(cc, kidx);
          if (kidx >= 0 && kidx < (int)ncm) atomicMin(&first[kidx], (u32)(v < 0xFFFFFFF0u ? v : 0xFFFFFFF0u));
        }
        const u32 fmin = wave_min_u32(fpos);
        if (fmin != 0xFFFFFFFFu) {
          const uint64_t owner = __ballot(fpos == fmin);
          const u32 fk = (u32)__shfl((int)fkind, __ffsll((unsigned long long)owner) - 1, 64);
          r.ok = false;
          r.panic = fk == KEY_PANIC;
        } else if (!whole) {
          r.ok = false;   // the list is cut inside a vote after every key decoded
        }
        __syncthreads();
        if (r.ok) {
          // pass 2: Certificate::verify's vote loop (messages.rs:198-208) stops at the first vote
          // whose name is already used (AuthorityReuse) or has no stake (UnknownAuthority); while
          // no error has occurred every earlier vote was inserted, so "used" = all earlier names.
          u32 err = 0xFFFFFFFFu;
          u32 err_kind = 0;
          for (uint64_t v = lane; v < V; v += 64) {
            const u32* kw = reinterpret_cast<const u32*>(a.v_pk + 32 * (vbase + v));
            u32 key[8];
            _Pragma("unroll") for (int k = 0; k < 8; ++k) key[k] = kw[k];
            const int kidx = committee_lookup(cm, key);
            const bool reused = kidx >= 0 && kidx < (int)ncm && first[kidx] < (u32)v;
            const bool unknown = member_stake(cc, kidx) == 0;
            if ((reused || unknown) && (u32)v < err) { err = (u32)v; err_kind = reused ? DAG_AUTHORITY_REUSE : DAG_UNKNOWN_AUTHORITY; }
          }
          const u32 emin = wave_min_u32(err);
          const bool mine = err == emin && emin != 0xFFFFFFFFu;
          const uint64_t owner = __ballot(mine);
          const u32 ek = (u32)__shfl((int)err_kind, owner ? __ffsll((unsigned long long)owner) - 1 : 0, 64);
          const uint64_t wsum = wave_sum_u64(weight);
          post = emin != 0xFFFFFFFFu ? ek : (wsum < cc.quorum ? DAG_REQUIRES_QUORUM : DAG_OK);
          vcount = (u32)V;
        }
      }
    }
    if (!r.ok) {
      flags |= MF_PARSE_ERR | (r.panic ? MF_PANIC : 0u);
      vcount = 0;   // (slots of a failed vote list keep v_msg = i or the host's zero fill: valid indices)
    } else {
      u32 z = 0;
      _Pragma("unroll") for (int k = 0; k < 8; ++k) z |= id[k];
      if (kind == MSG_CERTIFICATE && round == 0 && aidx >= 0 && z == 0) flags |= MF_GENESIS;
      if (a.gc_round > round) flags |= MF_TOO_OLD;
      if (astake == 0) flags |= MF_STAKE0;
    }
    _Pragma("unroll") for (int k = 0; k < 8; ++k) { eq_msg[k] = id[k]; eq_pk[k] = author[k]; dig[k] = cd[k]; }
    _Pragma("unroll") for (int k = 0; k < 16; ++k) eq_sig[k] = sig[k];
  } else if (kind == MSG_VOTE) {
    u32 id[8], origin[8], author[8], sg[16];
    r.bytes32(id);
    const uint64_t round = r.u64();
    r.key(origin);
    r.key(author);
    r.bytes64(sg);
    digest72(id, round, origin, dig);
    if (!r.ok) {
      flags |= MF_PARSE_ERR | (r.panic ? MF_PANIC : 0u);
    } else if (a.target.enabled && a.target.round > round) {
      post = DAG_TOO_OLD;   // Core::sanitize_vote (primary/src/core.rs:319-322)
    } else if (a.target.enabled && !(words_eq8(id, a.target.id) && words_eq8(origin, a.target.origin) &&
                                     round == a.target.round)) {
      post = DAG_UNEXPECTED_VOTE;   // core.rs:325-330
    } else if (member_stake(cc, committee_lookup(cm, author)) == 0) {
      post = DAG_UNKNOWN_AUTHORITY;   // Vote::verify (messages.rs:133-136)
    }
    _Pragma("unroll") for (int k = 0; k < 8; ++k) { eq_msg[k] = dig[k]; eq_pk[k] = author[k]; }
    _Pragma("unroll") for (int k = 0; k < 16; ++k) eq_sig[k] = sg[k];
  } else {
    post = (r.ok && variant == 3) ? DAG_UNEXPECTED_MESSAGE : DAG_SERIALIZATION;
  }
  if (lane == 0) {
    st_words(a.eq_msg + 32 * i, eq_msg, 8);
    st_words(a.eq_pk + 32 * i, eq_pk, 8);
    st_words(a.eq_sig + 64 * i, eq_sig, 16);
    st_words(a.cdig + 32 * i, cd, 8);
    if (a.digests && kind != MSG_HEADER) st_words(a.digests + 32 * i, dig, 8);
    a.rec[4 * i + 0] = kind | flags;
    a.rec[4 * i + 1] = post;
    a.rec[4 * i + 2] = vbase;
    a.rec[4 * i + 3] = hlen;
    a.rec_n[i] = vcount;
  }
}

// Header::digest of the gathered input, one lane per message (a header of 67 parents is 18 blocks)
__global__ __launch_bounds__(256) void k_header_digests(MsgArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m) return;
  const u32 r0 = a.rec[4 * i], kind = r0 & 255u;
  u32 match = 0;
  if ((kind == MSG_HEADER || kind == MSG_CERTIFICATE) && !(r0 & MF_PARSE_ERR)) {
    const uint8_t* hb = a.hashbuf + ((a.offsets[i] + 127) & ~(uint64_t)127) + 128 * i;
    u32 dg[8], id[8];
    sha512_trunc32_buf(hb, a.rec[4 * i + 3], dg);
    const u32* idw = reinterpret_cast<const u32*>(a.eq_msg + 32 * i);
    _Pragma("unroll") for (int k = 0; k < 8; ++k) id[k] = idw[k];
    match = words_eq8(dg, id) ? 1u : 0u;
    if (a.digests && kind == MSG_HEADER) st_words(a.digests + 32 * i, dg, 8);
  } else if (kind == MSG_HEADER && a.digests) {
    u32 z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    st_words(a.digests + 32 * i, z, 8);
  }
  a.hmatch[i] = match;
}

// code[i] in the reference's order:
//   header:      Serialization -> TooOld -> InvalidHeaderId -> UnknownAuthority -> MalformedHeader
//                -> InvalidSignature                        (core.rs:306-317, messages.rs:48-67)
//   certificate: Serialization -> TooOld -> genesis Ok -> (header checks) -> AuthorityReuse /
//                UnknownAuthority (first vote) -> CertificateRequiresQuorum -> InvalidSignature
//                                                            (core.rs:338-346, messages.rs:189-215)
//   vote:        Serialization -> TooOld -> UnexpectedVote -> UnknownAuthority -> InvalidSignature
// The shared vote-slot counter of a chunked call rounded up to a multiple of 64 (<= cap).  The
// skipped slots repeat the last vote parsed so far: a leaf launch over them then takes that
// vote's path (its key is cached), where stale slot bytes sent their uncached keys to the
// latency-bound list kernel, ~0.7 ms at the end of every chunked call (profiles/r05/wire_host.md).
// Their verdicts are never read.  One block of 64 threads.
__global__ void k_align_slots(uint32_t* v_total, uint32_t cap, uint8_t* __restrict__ v_pk, uint8_t* __restrict__ v_sig,
                              uint32_t* __restrict__ v_msg) {
  const uint32_t v0 = *v_total;
  const uint32_t a = (v0 + 63u) & ~63u, v = a < cap ? a : cap;
  if (v0 > 0 && v0 <= cap) {   // (a parse that overflowed the slots left the count above the cap)
    const uint4* pk = reinterpret_cast<const uint4*>(v_pk + 32 * (size_t)(v0 - 1));
    const uint4* sg = reinterpret_cast<const uint4*>(v_sig + 64 * (size_t)(v0 - 1));
    const uint4 p0 = pk[0], p1 = pk[1], s0 = sg[0], s1 = sg[1], s2 = sg[2], s3 = sg[3];
    const uint32_t mi = v_msg[v0 - 1];
    for (uint32_t j = v0 + threadIdx.x; j < v; j += blockDim.x) {
      uint4* dp = reinterpret_cast<uint4*>(v_pk + 32 * (size_t)j);
      uint4* ds = reinterpret_cast<uint4*>(v_sig + 64 * (size_t)j);
      dp[0] = p0;
      dp[1] = p1;
      ds[0] = s0;
      ds[1] = s1;
      ds[2] = s2;
      ds[3] = s3;
      v_msg[j] = mi;
    }
  }
  __syncthreads();   // every thread has read the count
  if (threadIdx.x == 0) *v_total = v;
}

__global__ void k_finalize_messages(const uint32_t* __restrict__ rec, const uint32_t* __restrict__ rec_n,
                                    const uint32_t* __restrict__ hmatch, const uint64_t* __restrict__ strict_bits,
                                    const uint64_t* __restrict__ leaf_bits, uint64_t m, int32_t* __restrict__ codes) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const u32 r0 = rec[4 * i], kind = r0 & 255u, post = rec[4 * i + 1], vbase = rec[4 * i + 2];
  const u32 vn = rec_n[i];
  const bool sig_ok = (strict_bits[i >> 6] >> (i & 63)) & 1;
  u32 code;
  if (kind == MSG_OTHER) {
    code = post;
  } else if (r0 & MF_PARSE_ERR) {
    code = (r0 & MF_PANIC) ? DAG_DECODE_PANIC : DAG_SERIALIZATION;
  } else if (kind == MSG_VOTE) {
    code = post != DAG_OK ? post : (sig_ok ? DAG_OK : DAG_INVALID_SIGNATURE);
  } else if (r0 & MF_TOO_OLD) {
    code = DAG_TOO_OLD;
  } else if (kind == MSG_CERTIFICATE && (r0 & MF_GENESIS)) {
    code = DAG_OK;
  } else if (!hmatch[i]) {
    code = DAG_INVALID_HEADER_ID;
  } else if (r0 & MF_STAKE0) {
    code = DAG_UNKNOWN_AUTHORITY;
  } else if (r0 & MF_WORKER_BAD) {
    code = DAG_MALFORMED_HEADER;
  } else if (!sig_ok) {
    code = DAG_INVALID_SIGNATURE;
  } else if (kind == MSG_HEADER) {
    code = DAG_OK;
  } else if (post != DAG_OK) {
    code = post;
  } else {
    bool all = true;
    for (u32 v = vbase; v < vbase + vn; ++v) all = all && ((leaf_bits[v >> 6] >> (v & 63)) & 1);
    code = all ? DAG_OK : DAG_INVALID_SIGNATURE;
  }
  codes[i] = (int32_t)code;
}

}  // namespace nwc
