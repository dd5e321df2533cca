/*
 * Third-party CPU baseline point for bench.py ("optional third-party point"):
 * OpenSSL 3's EVP Ed25519 single-signature verification (RFC 8032 / "ed25519ph-less" PureEdDSA)
 * on every host thread the box grants.  TEST/BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline
 * leg and tests/ load it; the product never does.
 *
 * Not dalek semantics: OpenSSL accepts non-canonical R/A encodings and small-order keys where
 * ed25519-dalek 1.0.1's verify_strict (crypto/src/lib.rs:186, the call Narwhal makes) rejects
 * them, and uses the cofactorless equation.  On honest triples — the bench workload — both say
 * "valid", which is all this point is used for: a speed reference from a widely deployed library.
 *
 * Messages are 32-byte Narwhal digests (crypto/src/lib.rs:30 Digest), one per triple.
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

typedef struct {
    const uint8_t *msgs, *pks, *sigs;
    uint8_t *out;
    size_t lo, hi;
} Range;

static int verify_one(EVP_MD_CTX *ctx, const uint8_t *m, const uint8_t *pk, const uint8_t *sig) {
    EVP_PKEY *key = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, pk, 32);
    if (!key) return 0;
    int ok = EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, key) == 1 &&
             EVP_DigestVerify(ctx, sig, 64, m, 32) == 1;
    EVP_PKEY_free(key);
    EVP_MD_CTX_reset(ctx);
    return ok;
}

static void *worker(void *arg) {
    Range *r = (Range *)arg;
    EVP_MD_CTX *ctx = EVP_MD_CTX_new();
    for (size_t i = r->lo; i < r->hi; i++)
        r->out[i] = ctx ? (uint8_t)verify_one(ctx, r->msgs + 32 * i, r->pks + 32 * i, r->sigs + 64 * i) : 0;
    EVP_MD_CTX_free(ctx);
    return NULL;
}

/* out[i] = 1 when OpenSSL accepts (msgs[i], pks[i], sigs[i]); returns the threads actually run. */
int ossl_ed25519_verify_many(const uint8_t *msgs, const uint8_t *pks, const uint8_t *sigs, size_t n,
                             uint8_t *out, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    if ((size_t)threads > n) threads = n ? (int)n : 1;
    pthread_t tid[1024];
    Range rg[1024];
    uint8_t started[1024] = {0};
    for (int t = 0; t < threads; t++) {
        rg[t] = (Range){msgs, pks, sigs, out, n * t / threads, n * (t + 1) / threads};
        if (t == 0) continue;
        if (pthread_create(&tid[t], NULL, worker, &rg[t]) == 0) started[t] = 1;
        else worker(&rg[t]);
    }
    worker(&rg[0]);
    for (int t = 1; t < threads; t++)
        if (started[t]) pthread_join(tid[t], NULL);
    return threads;
}
