/*
 * nwc_oracle.c -- CPU restatement of the reference's signature-and-digest hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it.  The product (narwhal_amd/libnwc.so) never
 * links, calls or falls back to it.
 *
 * Restated behaviour (reference = /root/reference, arithmetic in un-vendored crates
 * ed25519-dalek 1.0.1 / curve25519-dalek 3.x / ed25519 1.x / sha2 0.9, crypto/Cargo.toml:10;
 * semantics as specified in SURVEY.md Appendix A):
 *   orc_verify_strict      crypto::Signature::verify        crypto/src/lib.rs:200-204 (A.1-A.3)
 *   orc_verify_batch       crypto::Signature::verify_batch  crypto/src/lib.rs:206-219 (A.4)
 *   orc_leaf               per-signature bisection leaf     SURVEY.md A.5
 *   orc_sha512 / digest32  Sha512::digest(..)[..32]         worker/src/processor.rs:38
 *   orc_keygen / orc_sign  generate_keypair / Signature::new crypto/src/lib.rs:167-191 (fixtures)
 *
 * Field: radix 2^51, five u64 limbs, unsigned __int128 products (a serial-CPU design,
 * deliberately unlike the GPU's 10 x 25.5-bit signed limbs so the two are independent).
 * Pinned against tests/golden/ fixtures (RFC 8032 vectors, the reference's own test fixtures
 * reproduced offline, OpenSSL-checked valid signatures, hashlib SHA-512 vectors).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;
typedef uint8_t u8;
typedef uint32_t u32;

/* ================================================================ SHA-512 (FIPS 180-4) */
static const u64 K512[80] = {
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

static inline u64 ror64(u64 x, int n) { return (x >> n) | (x << (64 - n)); }

static void sha512_block(u64 st[8], const u8 *p) {
  u64 w[80];
  for (int i = 0; i < 16; ++i) {
    u64 v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | p[8 * i + j];
    w[i] = v;
  }
  for (int i = 16; i < 80; ++i) {
    u64 s0 = ror64(w[i - 15], 1) ^ ror64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    u64 s1 = ror64(w[i - 2], 19) ^ ror64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  u64 a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 80; ++i) {
    u64 t1 = h + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + w[i];
    u64 t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

typedef struct { u64 st[8]; u8 buf[128]; size_t nbuf; u64 total; } sha512_ctx;

static void sha512_init(sha512_ctx *c) {
  static const u64 iv[8] = {0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,
                            0xa54ff53a5f1d36f1ULL,0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,
                            0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL};
  memcpy(c->st, iv, sizeof iv); c->nbuf = 0; c->total = 0;
}
static void sha512_update(sha512_ctx *c, const u8 *p, size_t n) {
  c->total += n;
  if (c->nbuf) {
    size_t take = 128 - c->nbuf; if (take > n) take = n;
    memcpy(c->buf + c->nbuf, p, take); c->nbuf += take; p += take; n -= take;
    if (c->nbuf == 128) { sha512_block(c->st, c->buf); c->nbuf = 0; }
  }
  while (n >= 128) { sha512_block(c->st, p); p += 128; n -= 128; }
  if (n) { memcpy(c->buf, p, n); c->nbuf = n; }
}
static void sha512_final(sha512_ctx *c, u8 out[64]) {
  u64 bits = c->total * 8;
  u8 pad = 0x80; sha512_update(c, &pad, 1); c->total -= 1;
  u8 z = 0;
  while (c->nbuf != 112) { sha512_update(c, &z, 1); c->total -= 1; }
  u8 len[16] = {0};
  for (int i = 0; i < 8; ++i) len[15 - i] = (u8)(bits >> (8 * i));
  sha512_update(c, len, 16);
  for (int i = 0; i < 8; ++i) for (int j = 0; j < 8; ++j) out[8 * i + j] = (u8)(c->st[i] >> (56 - 8 * j));
}

void orc_sha512(const u8 *data, size_t n, u8 out[64]) {
  sha512_ctx c; sha512_init(&c); sha512_update(&c, data, n); sha512_final(&c, out);
}

/* Digest = SHA-512(bytes)[..32] over n messages laid out by offsets[n+1]. */
void orc_digest32_many(const u8 *data, const u64 *offsets, size_t n, u8 *out32) {
  for (size_t i = 0; i < n; ++i) {
    u8 h[64];
    orc_sha512(data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), h);
    memcpy(out32 + 32 * i, h, 32);
  }
}

/* ================================================================ GF(2^255-19), radix 2^51 */
typedef struct { u64 v[5]; } fe;
static const u64 M51 = (1ULL << 51) - 1;

static fe fe_c(u64 a, u64 b, u64 c, u64 d, u64 e) { fe r = {{a, b, c, d, e}}; return r; }
static fe fe_zero(void) { return fe_c(0, 0, 0, 0, 0); }
static fe fe_one(void) { return fe_c(1, 0, 0, 0, 0); }

static fe fe_carry(fe a) {
  u64 c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= M51; a.v[4] += c;
  c = a.v[4] >> 51; a.v[4] &= M51; a.v[0] += 19 * c;
  return a;
}
static fe fe_add(fe a, fe b) {
  fe r; for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i]; return fe_carry(r);
}
/* a - b: add 16p (limb-wise) so limbs stay non-negative for inputs < 2^54. */
static fe fe_sub(fe a, fe b) {
  fe r;
  r.v[0] = a.v[0] + 0x7FFFFFFFFFFED0ULL - b.v[0];
  for (int i = 1; i < 5; ++i) r.v[i] = a.v[i] + 0x7FFFFFFFFFFFF0ULL - b.v[i];
  return fe_carry(r);
}
static fe fe_neg(fe a) { return fe_sub(fe_zero(), a); }

static fe fe_mul(fe a, fe b) {
  u128 t[5];
  u64 b19[5]; for (int i = 0; i < 5; ++i) b19[i] = 19 * b.v[i];
  t[0] = (u128)a.v[0]*b.v[0] + (u128)a.v[1]*b19[4] + (u128)a.v[2]*b19[3] + (u128)a.v[3]*b19[2] + (u128)a.v[4]*b19[1];
  t[1] = (u128)a.v[0]*b.v[1] + (u128)a.v[1]*b.v[0] + (u128)a.v[2]*b19[4] + (u128)a.v[3]*b19[3] + (u128)a.v[4]*b19[2];
  t[2] = (u128)a.v[0]*b.v[2] + (u128)a.v[1]*b.v[1] + (u128)a.v[2]*b.v[0] + (u128)a.v[3]*b19[4] + (u128)a.v[4]*b19[3];
  t[3] = (u128)a.v[0]*b.v[3] + (u128)a.v[1]*b.v[2] + (u128)a.v[2]*b.v[1] + (u128)a.v[3]*b.v[0] + (u128)a.v[4]*b19[4];
  t[4] = (u128)a.v[0]*b.v[4] + (u128)a.v[1]*b.v[3] + (u128)a.v[2]*b.v[2] + (u128)a.v[3]*b.v[1] + (u128)a.v[4]*b.v[0];
  fe r; u64 c = 0;
  for (int i = 0; i < 5; ++i) { t[i] += c; r.v[i] = (u64)t[i] & M51; c = (u64)(t[i] >> 51); }
  r.v[0] += 19 * c;
  c = r.v[0] >> 51; r.v[0] &= M51; r.v[1] += c;
  return r;
}
static fe fe_sq(fe a) { return fe_mul(a, a); }
static fe fe_sqn(fe a, int n) { while (n--) a = fe_sq(a); return a; }

/* Canonical little-endian encoding (value mod p). */
static void fe_tobytes(u8 out[32], fe a) {
  a = fe_carry(fe_carry(a));
  /* now a < 2^255 + small; subtract p if a >= p */
  u64 q = (a.v[0] + 19) >> 51;
  q = (a.v[1] + q) >> 51; q = (a.v[2] + q) >> 51; q = (a.v[3] + q) >> 51; q = (a.v[4] + q) >> 51;
  a.v[0] += 19 * q;
  u64 c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= M51; a.v[4] += c;
  a.v[4] &= M51;
  u64 w[4];
  w[0] = a.v[0] | (a.v[1] << 51);
  w[1] = (a.v[1] >> 13) | (a.v[2] << 38);
  w[2] = (a.v[2] >> 26) | (a.v[3] << 25);
  w[3] = (a.v[3] >> 39) | (a.v[4] << 12);
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) out[8 * i + j] = (u8)(w[i] >> (8 * j));
}
/* Loads the low 255 bits (bit 255 ignored); values >= p are accepted (A.2 step 1). */
static fe fe_frombytes(const u8 in[32]) {
  u64 w[4];
  for (int i = 0; i < 4; ++i) { w[i] = 0; for (int j = 7; j >= 0; --j) w[i] = (w[i] << 8) | in[8 * i + j]; }
  fe r;
  r.v[0] = w[0] & M51;
  r.v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r.v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  r.v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r.v[4] = (w[3] >> 12) & M51;
  return r;
}
static int fe_eq(fe a, fe b) { u8 x[32], y[32]; fe_tobytes(x, a); fe_tobytes(y, b); return memcmp(x, y, 32) == 0; }
static int fe_iszero(fe a) { return fe_eq(a, fe_zero()); }
static int fe_isneg(fe a) { u8 x[32]; fe_tobytes(x, a); return x[0] & 1; }

/* a^((p-5)/8) = a^(2^252 - 3) */
static fe fe_pow22523(fe z) {
  fe z2 = fe_sq(z), z8 = fe_sqn(z2, 2), z9 = fe_mul(z, z8), z11 = fe_mul(z2, z9);
  fe z22 = fe_sq(z11), z_5_0 = fe_mul(z9, z22);
  fe z_10_0 = fe_mul(fe_sqn(z_5_0, 5), z_5_0);
  fe z_20_0 = fe_mul(fe_sqn(z_10_0, 10), z_10_0);
  fe z_40_0 = fe_mul(fe_sqn(z_20_0, 20), z_20_0);
  fe z_50_0 = fe_mul(fe_sqn(z_40_0, 10), z_10_0);
  fe z_100_0 = fe_mul(fe_sqn(z_50_0, 50), z_50_0);
  fe z_200_0 = fe_mul(fe_sqn(z_100_0, 100), z_100_0);
  fe z_250_0 = fe_mul(fe_sqn(z_200_0, 50), z_50_0);
  return fe_mul(fe_sqn(z_250_0, 2), z);
}
static fe fe_invert(fe z) {
  /* z^(p-2) = z^(2^255-21) = (z^(2^252-3))^8 * z^3 */
  fe t = fe_pow22523(z);
  t = fe_sqn(t, 3);
  return fe_mul(t, fe_mul(fe_sq(z), z));
}

static fe FE_D, FE_D2, FE_SQRTM1;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* ================================================================ group (extended coords) */
typedef struct { fe X, Y, Z, T; } ge;
typedef struct { fe YpX, YmX, Z, T2d; } ge_cached;

static ge ge_identity(void) { ge r = {fe_zero(), fe_one(), fe_one(), fe_zero()}; return r; }

static ge ge_add(ge p, ge q) {  /* add-2008-hwcd-3, a = -1 */
  fe a = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
  fe b = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
  fe c = fe_mul(fe_mul(p.T, q.T), FE_D2);
  fe d = fe_mul(p.Z, q.Z); d = fe_add(d, d);
  fe e = fe_sub(b, a), f = fe_sub(d, c), g = fe_add(d, c), h = fe_add(b, a);
  ge r = {fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
  return r;
}
static ge ge_dbl(ge p) {  /* dbl-2008-hwcd, a = -1 */
  fe a = fe_sq(p.X), b = fe_sq(p.Y), c = fe_sq(p.Z); c = fe_add(c, c);
  fe xy = fe_add(p.X, p.Y);
  fe e = fe_sub(fe_sub(fe_sq(xy), a), b);
  fe g = fe_sub(b, a);           /* D + B with D = -A */
  fe f = fe_sub(g, c);
  fe h = fe_neg(fe_add(a, b));   /* D - B */
  ge r = {fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
  return r;
}
static ge ge_neg(ge p) { p.X = fe_neg(p.X); p.T = fe_neg(p.T); return p; }
static int ge_is_identity(ge p) { return fe_iszero(p.X) && fe_eq(p.Y, p.Z); }
static int ge_eq(ge p, ge q) {  /* dalek EdwardsPoint ct_eq: X1Z2 == X2Z1 && Y1Z2 == Y2Z1 */
  return fe_eq(fe_mul(p.X, q.Z), fe_mul(q.X, p.Z)) && fe_eq(fe_mul(p.Y, q.Z), fe_mul(q.Y, p.Z));
}
static int ge_is_small_order(ge p) { return ge_is_identity(ge_dbl(ge_dbl(ge_dbl(p)))); }

static void ge_tobytes(u8 out[32], ge p) {
  fe zi = fe_invert(p.Z);
  fe x = fe_mul(p.X, zi), y = fe_mul(p.Y, zi);
  fe_tobytes(out, y);
  out[31] |= (u8)(fe_isneg(x) << 7);
}

/* curve25519-dalek CompressedEdwardsY::decompress. Returns 1 on success. */
static int ge_decompress(ge *r, const u8 s[32]) {
  fe y = fe_frombytes(s), z = fe_one();
  fe yy = fe_sq(y);
  fe u = fe_sub(yy, z);
  fe v = fe_add(fe_mul(yy, FE_D), z);
  /* sqrt_ratio_i(u, v) */
  fe v3 = fe_mul(fe_sq(v), v);
  fe v7 = fe_mul(fe_sq(v3), v);
  fe x = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  fe check = fe_mul(v, fe_sq(x));
  int correct = fe_eq(check, u);
  int flipped = fe_eq(check, fe_neg(u));
  int flipped_i = fe_eq(check, fe_mul(fe_neg(u), FE_SQRTM1));
  if (flipped || flipped_i) x = fe_mul(x, FE_SQRTM1);
  if (fe_isneg(x)) x = fe_neg(x);
  if (!(correct || flipped)) return 0;
  if (s[31] >> 7) x = fe_neg(x);   /* even when x == 0 (accepted) */
  r->X = x; r->Y = y; r->Z = z; r->T = fe_mul(x, y);
  return 1;
}

/* ================================================================ scalars mod l */
/* l = 2^252 + 27742317777372353535851937790883648493, little-endian 64-bit words */
static const u64 L_W[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};

/* r = x mod l for a 512-bit little-endian x (Scalar::from_hash / from_bytes_mod_order_wide). */
static void sc_reduce512(u8 out[32], const u8 in[64]) {
  /* schoolbook: process bits from the top, r = 2r + bit, r < l (simple and independent) */
  u64 r[4] = {0, 0, 0, 0};
  for (int bit = 511; bit >= 0; --bit) {
    u64 carry = r[3] >> 63;
    r[3] = (r[3] << 1) | (r[2] >> 63); r[2] = (r[2] << 1) | (r[1] >> 63);
    r[1] = (r[1] << 1) | (r[0] >> 63); r[0] = (r[0] << 1) | ((in[bit >> 3] >> (bit & 7)) & 1);
    /* if r >= l: r -= l (r < 2l < 2^254, carry is always 0) */
    (void)carry;
    int ge_l = 0;
    for (int i = 3; i >= 0; --i) { if (r[i] != L_W[i]) { ge_l = r[i] > L_W[i]; break; } if (i == 0) ge_l = 1; }
    if (ge_l) {
      u64 br = 0;
      for (int i = 0; i < 4; ++i) { u128 d = (u128)r[i] - L_W[i] - br; r[i] = (u64)d; br = (u64)(d >> 64) & 1; }
    }
  }
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) out[8 * i + j] = (u8)(r[i] >> (8 * j));
}
static int sc_lt_l(const u8 s[32]) {
  for (int i = 31; i >= 0; --i) {
    u8 lb = (u8)(L_W[i >> 3] >> (8 * (i & 7)));
    if (s[i] != lb) return s[i] < lb;
  }
  return 0;
}
/* A.1: ed25519 1.x Signature::from_bytes + dalek check_scalar => s < l */
static int sig_scalar_ok(const u8 sig[64]) {
  if (sig[63] & 0xE0) return 0;
  if ((sig[63] & 0xF0) == 0) return 1;
  return sc_lt_l(sig + 32);
}
/* (a*b + c) mod l for 32-byte little-endian scalars (signing only) */
static void sc_muladd(u8 out[32], const u8 a[32], const u8 b[32], const u8 c[32]) {
  u8 prod[64] = {0};
  u64 t[8] = {0};
  u64 aw[4], bw[4], cw[4];
  for (int i = 0; i < 4; ++i) { aw[i] = bw[i] = cw[i] = 0;
    for (int j = 7; j >= 0; --j) { aw[i] = (aw[i] << 8) | a[8*i+j]; bw[i] = (bw[i] << 8) | b[8*i+j]; cw[i] = (cw[i] << 8) | c[8*i+j]; } }
  for (int i = 0; i < 4; ++i) {
    u128 carry = 0;
    for (int j = 0; j < 4; ++j) { u128 v = (u128)aw[i] * bw[j] + t[i + j] + carry; t[i + j] = (u64)v; carry = v >> 64; }
    t[i + 4] = (u64)carry;
  }
  u128 carry = 0;
  for (int i = 0; i < 8; ++i) { u128 v = (u128)t[i] + (i < 4 ? cw[i] : 0) + carry; t[i] = (u64)v; carry = v >> 64; }
  for (int i = 0; i < 8; ++i) for (int j = 0; j < 8; ++j) prod[8 * i + j] = (u8)(t[i] >> (8 * j));
  sc_reduce512(out, prod);
}

/* ================================================================ scalar multiplication */
static ge ge_scalarmult(const u8 k[32], ge p) {  /* variable-time double-and-add, top-down */
  ge r = ge_identity();
  for (int bit = 255; bit >= 0; --bit) {
    r = ge_dbl(r);
    if ((k[bit >> 3] >> (bit & 7)) & 1) r = ge_add(r, p);
  }
  return r;
}

/* width-w NAF of a 256-bit scalar (digits odd, |d| < 2^(w-1), nonzero digits >= w apart) */
static void slide(signed char naf[257], const u8 k[32], int w) {
  /* Generic, clear w-NAF using a mutable big integer (little-endian u64 words). */
  u64 x[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) for (int j = 7; j >= 0; --j) x[i] = (x[i] << 8) | k[8 * i + j];
  memset(naf, 0, 257);
  int pos = 0;
  const int W = 1 << w, H = 1 << (w - 1);
  while (pos < 257) {
    const u64 nz = x[0] | x[1] | x[2] | x[3] | x[4];   /* u64: an int truncation ended the NAF early */
    if (!nz) break;
    if (x[0] & 1) {
      int d = (int)(x[0] & (u64)(W - 1));
      if (d >= H) d -= W;
      naf[pos] = (signed char)d;
      /* x -= d */
      if (d > 0) { u64 br = (u64)d; for (int i = 0; i < 5 && br; ++i) { u64 o = x[i]; x[i] -= br; br = o < br; } }
      else { u64 cr = (u64)(-d); for (int i = 0; i < 5 && cr; ++i) { u64 o = x[i]; x[i] += cr; cr = x[i] < o; } }
    }
    /* x >>= 1 */
    for (int i = 0; i < 4; ++i) x[i] = (x[i] >> 1) | (x[i + 1] << 63);
    x[4] >>= 1;
    ++pos;
  }
}

static ge B_ODD[64];   /* odd multiples 1B..127B of the basepoint */
static ge BASE;

/* a*A + b*B, variable time (dalek vartime_double_scalar_mul_basepoint semantics:
   the result is the group element; the algorithm is irrelevant to the verdict). */
static ge ge_double_scalarmult_vartime(const u8 a[32], ge A, const u8 b[32]) {
  signed char an[257], bn[257];
  slide(an, a, 5);
  slide(bn, b, 8);
  ge ai[8];
  ai[0] = A;
  ge a2 = ge_dbl(A);
  for (int i = 1; i < 8; ++i) ai[i] = ge_add(ai[i - 1], a2);
  int top = 256;
  while (top >= 0 && !an[top] && !bn[top]) --top;
  ge r = ge_identity();
  for (int i = top; i >= 0; --i) {
    r = ge_dbl(r);
    if (an[i] > 0) r = ge_add(r, ai[an[i] / 2]);
    else if (an[i] < 0) r = ge_add(r, ge_neg(ai[(-an[i]) / 2]));
    if (bn[i] > 0) r = ge_add(r, B_ODD[bn[i] / 2]);
    else if (bn[i] < 0) r = ge_add(r, ge_neg(B_ODD[(-bn[i]) / 2]));
  }
  return r;
}

static void init_consts(void) {
  /* d = -121665/121666 */
  fe n = fe_c(121665, 0, 0, 0, 0), dd = fe_c(121666, 0, 0, 0, 0);
  FE_D = fe_mul(fe_neg(n), fe_invert(dd));
  FE_D2 = fe_add(FE_D, FE_D);
  /* sqrt(-1) = 2^((p-1)/4) */
  fe two = fe_c(2, 0, 0, 0, 0);
  /* (p-1)/4 = 2^253 - 5: compute 2^(2^253-5) = 2^(2^253-8) * 2^3 = (2^(2^250-1))^8 * 8 */
  /* simpler: pow22523(2) = 2^(2^252-3); square it: 2^(2^253-6); times 2: 2^(2^253-5) */
  fe t = fe_pow22523(two);
  FE_SQRTM1 = fe_mul(fe_sq(t), two);
  u8 by[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
               0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
  ge_decompress(&BASE, by);
  ge b2 = ge_dbl(BASE);
  B_ODD[0] = BASE;
  for (int i = 1; i < 64; ++i) B_ODD[i] = ge_add(B_ODD[i - 1], b2);
}
static void ensure_init(void) { pthread_once(&g_once, init_consts); }

/* ================================================================ verify (A.3 - A.5) */
/* crypto::Signature::verify -> verify_strict. 1 = Ok, 0 = Err. */
int orc_verify_strict(const u8 msg32[32], const u8 pk[32], const u8 sig[64]) {
  ensure_init();
  if (!sig_scalar_ok(sig)) return 0;
  ge A, R;
  if (!ge_decompress(&A, pk)) return 0;
  if (!ge_decompress(&R, sig)) return 0;
  if (ge_is_small_order(R) || ge_is_small_order(A)) return 0;
  u8 h[64], k[32];
  sha512_ctx c; sha512_init(&c);
  sha512_update(&c, sig, 32); sha512_update(&c, pk, 32); sha512_update(&c, msg32, 32);
  sha512_final(&c, h);
  sc_reduce512(k, h);
  ge Rp = ge_double_scalarmult_vartime(k, ge_neg(A), sig + 32);
  return ge_eq(Rp, R);
}

/* l * P != O: P has a non-zero 8-torsion component (curve25519-dalek 3 is_torsion_free, negated) */
static const u8 L_BYTES[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9,
                               0xde, 0x14, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};
static int ge_has_torsion(ge p) { return !ge_is_identity(ge_scalarmult(L_BYTES, p)); }

/* One vote of dalek 1.0.1 verify_batch (crypto/src/lib.rs:206-219).  dalek checks
     -(sum z_i s_i mod l) B + sum z_i R_i + sum (z_i k_i mod l) A_i == O
   with random 128-bit z_i.  With z_i k_i = (z_i k_i mod l) + q_i l the sum is
   -sum z_i e_i - sum q_i (l A_i), e_i = s_i B - R_i - k_i A_i, and l A_i = l T_i for the 8-torsion
   component T_i of A_i.  Class: -1 = parse/decode failure, 2 = e_i has a prime-order component
   (Err w.p. 1 - 2^-125), 1 = randomized (e_i pure torsion, and e_i != O or T_i != O: the verdict
   depends on z_i and q_i = floor(z_i k_i / l)), 0 = deterministic Ok. */
int orc_vote_class(const u8 msg32[32], const u8 pk[32], const u8 sig[64]) {
  ensure_init();
  if (!sig_scalar_ok(sig)) return -1;
  ge A, R;
  if (!ge_decompress(&A, pk)) return -1;
  if (!ge_decompress(&R, sig)) return -1;
  u8 h[64], k[32];
  sha512_ctx c; sha512_init(&c);
  sha512_update(&c, sig, 32); sha512_update(&c, pk, 32); sha512_update(&c, msg32, 32);
  sha512_final(&c, h);
  sc_reduce512(k, h);
  ge Rp = ge_double_scalarmult_vartime(k, ge_neg(A), sig + 32);
  ge e = ge_add(Rp, ge_neg(R));
  if (!ge_is_small_order(e)) return 2;
  if (!ge_is_identity(e) || ge_has_torsion(A)) return 1;
  return 0;
}

/* A.5 leaf = dalek verify_batch([vote]) decided deterministically: parses, decodes,
   s*B - R - k*A == identity (cofactorless) and A torsion-free.  The randomized domain is Err. */
int orc_leaf(const u8 msg32[32], const u8 pk[32], const u8 sig[64]) {
  return orc_vote_class(msg32, pk, sig) == 0;
}

/* crypto::Signature::verify_batch: one digest, n votes (pk_i, sig_i). Deterministic build
   verdict: Ok iff every leaf is Ok; empty -> Ok. bad (nullable) gets one byte per vote. */
int orc_verify_batch(const u8 msg32[32], const u8 *pks, const u8 *sigs, size_t n, u8 *bad) {
  int ok = 1;
  for (size_t i = 0; i < n; ++i) {
    int l = orc_leaf(msg32, pks + 32 * i, sigs + 64 * i);
    if (bad) bad[i] = (u8)!l;
    ok &= l;
  }
  return ok;
}

/* ---------------------------------------------------------------- dalek batch algorithm
 * ed25519-dalek 1.0.1 `verify_batch` (features = ["batch"], crypto/Cargo.toml:10) restated as the
 * CPU baseline for certificates: parse every signature and key (any failure ->
 * Err), hram_i = H(R_i || A_i || M) mod l, random 128-bit z_i, and one multiscalar multiplication
 *     (-sum z_i s_i) B + sum z_i R_i + sum (z_i hram_i) A_i  == identity   (cofactorless)
 * by Straus with width-5 NAFs and per-point tables of odd multiples (curve25519-dalek 3's vartime
 * Straus, used below 190 points).  dalek draws z_i from a merlin transcript finalised with
 * thread_rng; here a seeded xorshift supplies them -- the verdict is the same on the deterministic
 * domain (Ok iff every leaf holds, A.4), which is what the baseline runs on. */
static void sc_neg(u8 out[32], const u8 a[32]) {
  static const u8 LM1[32] = {0xec, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9,
                             0xde, 0x14, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};   /* l - 1 */
  static const u8 Z[32] = {0};
  sc_muladd(out, a, LM1, Z);
}
int orc_verify_batch_straus(const u8 msg32[32], const u8 *pks, const u8 *sigs, size_t n, u64 seed) {
  ensure_init();
  if (n == 0) return 1;
  const size_t np = 2 * n + 1;
  ge *tab = (ge *)malloc(sizeof(ge) * 8 * np);
  signed char (*naf)[257] = (signed char (*)[257])malloc(257 * np);
  u8 bsc[32] = {0};
  static const u8 Z[32] = {0};
  int ok = 1;
  u64 x = seed ^ 0x9E3779B97F4A7C15ULL;
  for (size_t i = 0; i < n && ok; ++i) {
    const u8 *pk = pks + 32 * i, *sig = sigs + 64 * i;
    ge A, R;
    if (!sig_scalar_ok(sig) || !ge_decompress(&A, pk) || !ge_decompress(&R, sig)) { ok = 0; break; }
    u8 hh[64], hram[32], z[32] = {0}, zh[32], acc[32];
    sha512_ctx c; sha512_init(&c);
    sha512_update(&c, sig, 32); sha512_update(&c, pk, 32); sha512_update(&c, msg32, 32);
    sha512_final(&c, hh);
    sc_reduce512(hram, hh);
    for (int k = 0; k < 16; ++k) {   /* 128-bit z_i (xorshift64*) */
      x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
      z[k] = (u8)((x * 0x2545F4914F6CDD1DULL) >> 56);
    }
    sc_muladd(zh, z, hram, Z);
    sc_muladd(acc, z, sig + 32, bsc);
    memcpy(bsc, acc, 32);
    slide(naf[1 + 2 * i], z, 5);
    slide(naf[2 + 2 * i], zh, 5);
    ge pts[2] = {R, A};
    for (int q = 0; q < 2; ++q) {
      ge *t = tab + 8 * (1 + 2 * i + q);
      t[0] = pts[q];
      ge p2 = ge_dbl(pts[q]);
      for (int k = 1; k < 8; ++k) t[k] = ge_add(t[k - 1], p2);
    }
  }
  if (ok) {
    u8 nb[32];
    sc_neg(nb, bsc);
    slide(naf[0], nb, 5);
    ge *t = tab;
    t[0] = BASE;
    ge p2 = ge_dbl(BASE);
    for (int k = 1; k < 8; ++k) t[k] = ge_add(t[k - 1], p2);
    ge r = ge_identity();
    for (int bit = 256; bit >= 0; --bit) {
      r = ge_dbl(r);
      for (size_t j = 0; j < np; ++j) {
        const int d = naf[j][bit];
        if (d > 0) r = ge_add(r, tab[8 * j + d / 2]);
        else if (d < 0) r = ge_add(r, ge_neg(tab[8 * j + (-d) / 2]));
      }
    }
    ok = ge_is_identity(r);
  }
  free(tab);
  free(naf);
  return ok;
}

/* dalek 1.0.1 verify_batch's equation for GIVEN 128-bit z_i (16 little-endian bytes each), term
   by term as the crate states it:  -(sum z_i s_i mod l) B + sum z_i R_i + sum (z_i k_i mod l) A_i
   == O (plain double-and-add per term; the test reference for orc_batch_z8).  1 = holds. */
int orc_batch_eq_z(const u8 msg32[32], const u8 *pks, const u8 *sigs, size_t n, const u8 *zs) {
  ensure_init();
  static const u8 Z[32] = {0};
  u8 bsc[32] = {0};
  ge acc = ge_identity();
  for (size_t i = 0; i < n; ++i) {
    const u8 *pk = pks + 32 * i, *sig = sigs + 64 * i;
    ge A, R;
    if (!sig_scalar_ok(sig) || !ge_decompress(&A, pk) || !ge_decompress(&R, sig)) return 0;
    u8 hh[64], k[32], z[32] = {0}, zk[32], t[32];
    sha512_ctx c; sha512_init(&c);
    sha512_update(&c, sig, 32); sha512_update(&c, pk, 32); sha512_update(&c, msg32, 32);
    sha512_final(&c, hh);
    sc_reduce512(k, hh);
    memcpy(z, zs + 16 * i, 16);
    sc_muladd(zk, z, k, Z);
    sc_muladd(t, z, sig + 32, bsc);
    memcpy(bsc, t, 32);
    acc = ge_add(acc, ge_add(ge_scalarmult(z, R), ge_scalarmult(zk, A)));
  }
  u8 nb[32];
  sc_neg(nb, bsc);
  acc = ge_add(acc, ge_scalarmult(nb, BASE));
  return ge_is_identity(acc);
}

/* j in 0..7 with p == [j] G8 (G8: the order-8 point with y = 26e8958f..6d53fc05, x even), -1 if
   p is not in E[8] */
static int torsion_dlog(ge p) {
  static const u8 G8[32] = {0x26, 0xe8, 0x95, 0x8f, 0xc2, 0xb2, 0x27, 0xb0, 0x45, 0xc3, 0xf4, 0x89, 0xf2, 0xef, 0x98, 0xf0,
                            0xd5, 0xdf, 0xac, 0x05, 0xd3, 0xc6, 0x33, 0x39, 0xb1, 0x38, 0x02, 0x88, 0x6d, 0x53, 0xfc, 0x05};
  ge g, acc = ge_identity();
  if (!ge_decompress(&g, G8)) return -1;
  for (int j = 0; j < 8; ++j) {
    if (ge_eq(acc, p)) return j;
    acc = ge_add(acc, g);
  }
  return -1;
}

/* The same equation for the same z_i, evaluated in E[8] = Z/8 as the GPU resolves it
   (narwhal_amd/csrc/resolve.h): -sum (z_i e_i + q_i (l A_i)) with e_i = s_i B - R_i - k_i A_i and
   z_i k_i = (z_i k_i mod l) + q_i l.  A vote that does not parse or decode, or whose e_i is not
   pure torsion, fails it (decided: Err w.p. 1 - 2^-125); otherwise e_i = [a_i] G8, l A_i = [b_i] G8
   and the equation holds iff sum (z_i a_i + q_i b_i) = 0 mod 8 (q_i mod 8 = (z_i k_i - (z_i k_i
   mod l)) / l mod 8 = 5 ((z_i k_i mod 8) - (z_i k_i mod l mod 8)) mod 8, since 1/l = 5 mod 8). */
int orc_batch_z8(const u8 msg32[32], const u8 *pks, const u8 *sigs, size_t n, const u8 *zs) {
  ensure_init();
  static const u8 Z[32] = {0};
  unsigned total = 0;
  for (size_t i = 0; i < n; ++i) {
    const u8 *pk = pks + 32 * i, *sig = sigs + 64 * i;
    ge A, R;
    if (!sig_scalar_ok(sig) || !ge_decompress(&A, pk) || !ge_decompress(&R, sig)) return 0;
    u8 hh[64], k[32], z[32] = {0}, zk[32];
    sha512_ctx c; sha512_init(&c);
    sha512_update(&c, sig, 32); sha512_update(&c, pk, 32); sha512_update(&c, msg32, 32);
    sha512_final(&c, hh);
    sc_reduce512(k, hh);
    ge e = ge_add(ge_double_scalarmult_vartime(k, ge_neg(A), sig + 32), ge_neg(R));
    if (!ge_is_small_order(e)) return 0;
    memcpy(z, zs + 16 * i, 16);
    sc_muladd(zk, z, k, Z);
    const unsigned z8 = z[0] & 7u, q8 = (5u * ((z8 * (k[0] & 7u) + 8u - (zk[0] & 7u)) & 7u)) & 7u;
    const int de = torsion_dlog(e), dl = torsion_dlog(ge_scalarmult(L_BYTES, A));
    if (de < 0 || dl < 0) return 0;
    total += z8 * (unsigned)de + q8 * (unsigned)dl;
  }
  return (total & 7u) == 0;
}

/* orc_batch_eq_z (which = 0) or orc_batch_z8 (which = 1) over m certificates (voffs, m + 1
   offsets; zs: 16 bytes per vote), out[c] = 1 if the equation holds */
void orc_batch_z_many(const u8 *digests, const u32 *voffs, const u8 *pks, const u8 *sigs, const u8 *zs, size_t m,
                      u8 *out, int which) {
  for (size_t c = 0; c < m; ++c) {
    const u32 a = voffs[c], n = voffs[c + 1] - a;
    out[c] = (u8)(which ? orc_batch_z8(digests + 32 * c, pks + 32 * (size_t)a, sigs + 64 * (size_t)a, n, zs + 16 * (size_t)a)
                        : orc_batch_eq_z(digests + 32 * c, pks + 32 * (size_t)a, sigs + 64 * (size_t)a, n, zs + 16 * (size_t)a));
  }
}

/* ================================================================ signing (fixtures, data) */
void orc_public_key(const u8 seed[32], u8 pk[32]) {
  ensure_init();
  u8 h[64]; orc_sha512(seed, 32, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  ge_tobytes(pk, ge_scalarmult(h, BASE));
}
void orc_sign(const u8 seed[32], const u8 *msg, size_t mlen, u8 sig[64]) {
  ensure_init();
  u8 h[64]; orc_sha512(seed, 32, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  u8 pk[32]; ge_tobytes(pk, ge_scalarmult(h, BASE));
  u8 rh[64], r[32];
  sha512_ctx c; sha512_init(&c); sha512_update(&c, h + 32, 32); sha512_update(&c, msg, mlen); sha512_final(&c, rh);
  sc_reduce512(r, rh);
  ge_tobytes(sig, ge_scalarmult(r, BASE));
  u8 kh[64], k[32];
  sha512_init(&c); sha512_update(&c, sig, 32); sha512_update(&c, pk, 32); sha512_update(&c, msg, mlen); sha512_final(&c, kh);
  sc_reduce512(k, kh);
  sc_muladd(sig + 32, k, h, r);
}

/* ================================================================ multithreaded drivers */
typedef struct {
  int kind;  /* 0 strict, 1 leaf, 2 batch-certs, 3 digest, 4 batch-certs (Straus), 5 vote class + 1 */
  const u8 *msgs, *pks, *sigs; const u64 *offsets; const u32 *voffs; const u8 *data;
  u8 *out, *out2; size_t lo, hi;
} job_t;

static void *worker(void *p) {
  job_t *j = (job_t *)p;
  for (size_t i = j->lo; i < j->hi; ++i) {
    if (j->kind == 0) j->out[i] = (u8)orc_verify_strict(j->msgs + 32 * i, j->pks + 32 * i, j->sigs + 64 * i);
    else if (j->kind == 1) j->out[i] = (u8)orc_leaf(j->msgs + 32 * i, j->pks + 32 * i, j->sigs + 64 * i);
    else if (j->kind == 5) j->out[i] = (u8)(orc_vote_class(j->msgs + 32 * i, j->pks + 32 * i, j->sigs + 64 * i) + 1);
    else if (j->kind == 2) {
      u32 a = j->voffs[i], b = j->voffs[i + 1];
      j->out[i] = (u8)orc_verify_batch(j->msgs + 32 * i, j->pks + 32 * (size_t)a, j->sigs + 64 * (size_t)a, b - a,
                                       j->out2 ? j->out2 + a : NULL);
    } else if (j->kind == 4) {
      u32 a = j->voffs[i], b = j->voffs[i + 1];
      j->out[i] = (u8)orc_verify_batch_straus(j->msgs + 32 * i, j->pks + 32 * (size_t)a, j->sigs + 64 * (size_t)a,
                                              b - a, (u64)i * 0x100000001B3ULL + 1);
    } else {
      u8 h[64];
      orc_sha512(j->data + j->offsets[i], (size_t)(j->offsets[i + 1] - j->offsets[i]), h);
      memcpy(j->out + 32 * i, h, 32);
    }
  }
  return NULL;
}

static void run_jobs(job_t proto, size_t n, int nthreads) {
  ensure_init();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 512) nthreads = 512;
  pthread_t th[512]; job_t jobs[512];
  size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
  int used = 0;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = proto; jobs[t].lo = (size_t)t * per; jobs[t].hi = jobs[t].lo + per;
    if (jobs[t].hi > n) jobs[t].hi = n;
    if (jobs[t].lo >= jobs[t].hi) break;
    pthread_create(&th[t], NULL, worker, &jobs[t]); ++used;
  }
  for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
}

void orc_verify_strict_many(const u8 *msgs, const u8 *pks, const u8 *sigs, size_t n, u8 *out, int nthreads) {
  job_t j; memset(&j, 0, sizeof j); j.kind = 0; j.msgs = msgs; j.pks = pks; j.sigs = sigs; j.out = out;
  run_jobs(j, n, nthreads);
}
void orc_leaf_many(const u8 *msgs, const u8 *pks, const u8 *sigs, size_t n, u8 *out, int nthreads) {
  job_t j; memset(&j, 0, sizeof j); j.kind = 1; j.msgs = msgs; j.pks = pks; j.sigs = sigs; j.out = out;
  run_jobs(j, n, nthreads);
}
/* orc_vote_class of n triples, stored + 1 (0 = parse/decode failure, 1 = ok, 2 = randomized, 3 = err) */
void orc_vote_class_many(const u8 *msgs, const u8 *pks, const u8 *sigs, size_t n, u8 *out, int nthreads) {
  job_t j; memset(&j, 0, sizeof j); j.kind = 5; j.msgs = msgs; j.pks = pks; j.sigs = sigs; j.out = out;
  run_jobs(j, n, nthreads);
}
/* m certificates: digests[32*m], vote ranges voffs[m+1] into pks/sigs; cert_ok[m], bad[votes] */
void orc_verify_batch_many(const u8 *digests, const u32 *voffs, const u8 *pks, const u8 *sigs, size_t m,
                           u8 *cert_ok, u8 *bad, int nthreads) {
  job_t j; memset(&j, 0, sizeof j); j.kind = 2; j.msgs = digests; j.voffs = voffs; j.pks = pks; j.sigs = sigs;
  j.out = cert_ok; j.out2 = bad;
  run_jobs(j, m, nthreads);
}
/* m certificates through the dalek batch algorithm (CPU baseline of config 3): cert_ok[m] */
void orc_verify_batch_straus_many(const u8 *digests, const u32 *voffs, const u8 *pks, const u8 *sigs, size_t m,
                                  u8 *cert_ok, int nthreads) {
  job_t j; memset(&j, 0, sizeof j); j.kind = 4; j.msgs = digests; j.voffs = voffs; j.pks = pks; j.sigs = sigs;
  j.out = cert_ok;
  run_jobs(j, m, nthreads);
}
void orc_digest32_many_mt(const u8 *data, const u64 *offsets, size_t n, u8 *out32, int nthreads) {
  job_t j; memset(&j, 0, sizeof j); j.kind = 3; j.data = data; j.offsets = offsets; j.out = out32;
  run_jobs(j, n, nthreads);
}

typedef struct { const u8 *seeds; const u8 *msgs; size_t mlen; u8 *pks; u8 *sigs; size_t lo, hi; } sjob_t;
static void *sworker(void *p) {
  sjob_t *j = (sjob_t *)p;
  for (size_t i = j->lo; i < j->hi; ++i) {
    orc_public_key(j->seeds + 32 * i, j->pks + 32 * i);
    orc_sign(j->seeds + 32 * i, j->msgs + j->mlen * i, j->mlen, j->sigs + 64 * i);
  }
  return NULL;
}
/* keygen + sign n (seed_i, msg_i) pairs in parallel (fixtures / CPU-side data only) */
void orc_keygen_sign_many(const u8 *seeds, const u8 *msgs, size_t mlen, size_t n, u8 *pks, u8 *sigs, int nthreads) {
  ensure_init();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 512) nthreads = 512;
  pthread_t th[512]; sjob_t jobs[512];
  size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
  int used = 0;
  for (int t = 0; t < nthreads; ++t) {
    sjob_t jj = {seeds, msgs, mlen, pks, sigs, (size_t)t * per, (size_t)t * per + per};
    if (jj.hi > n) jj.hi = n;
    if (jj.lo >= jj.hi) break;
    jobs[t] = jj; pthread_create(&th[t], NULL, sworker, &jobs[t]); ++used;
  }
  for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
}
