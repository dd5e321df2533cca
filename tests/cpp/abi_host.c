/* A plain C host of libnwc.so -- what the Rust `crypto` shim does, with no
 * Python or torch in the process: init, Signature::verify, Signature::verify_batch with its
 * bad-vote bitmap, and the worker's batch digest.
 *
 * stdin, one request per line (hex fields):
 *   S <msg32> <pk32> <sig64>            -> "S <rc>"                 (nwc_verify_strict)
 *   B <msg32> <n> <pk32 sig64> x n      -> "B <rc> <bad bitmap>"    (nwc_verify_batch)
 *   D <data>                            -> "D <digest32>"           (nwc_sha512_trunc32_many)
 *   V <n>, then n lines <msg32 pk32 sig64>  -> "V <rc> <bitmap>"     (nwc_verify_strict_many)
 *   C <m> <offsets m+1>, then offsets[m] vote lines <digest-index pk32 sig64> and m digest lines
 *                                       -> "C <rc> <cert bitmap> <bad bitmap>" (nwc_verify_batch_many)
 *   X <threads> <rounds>                -> "X <mismatches>": every B request so far re-run from
 *                                          that many concurrent host threads, results compared
 *   K <n> <pk32> x n                    -> "K <rc>"                 (nwc_set_committee; n = 0 clears)
 *   L <calls> <warm> <msg32> <n> <pk32 sig64> x n
 *                                       -> "L <rc> <first> <second> <p50> <p90> <p99> <p99.9> <max> <mean>"
 *                                          per-call latency (us) of nwc_verify_batch timed in C;
 *                                          percentiles over calls warm..calls-1
 *   Z                                   -> a heap read one byte out of bounds (sanitizer self-check)
 * Built by __graft_entry__.build() into tests/cpp/build/abi_host (and, host code under
 * AddressSanitizer + UBSan against a sanitized libnwc, abi_host_asan); run by
 * tests/test_gpu_abi_host.py.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nwc.h"

static int cmp_double(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return (x > y) - (x < y);
}

/* B requests kept for the X (concurrency) command */
typedef struct {
  unsigned char m[32];
  unsigned char* pks;
  unsigned char* sigs;
  size_t n;
  int rc;
  unsigned char* bad;
} breq;
static breq g_b[4096];
static size_t g_nb;
static int g_rounds;

static void* worker(void* arg) {
  long bad_count = 0;
  (void)arg;
  for (int r = 0; r < g_rounds; ++r) {
    for (size_t i = 0; i < g_nb; ++i) {
      const breq* q = &g_b[i];
      unsigned char* bad = calloc(q->n / 8 + 1, 1);
      const int rc = nwc_verify_batch(q->m, q->pks, q->sigs, q->n, bad);
      if (rc != q->rc || memcmp(bad, q->bad, (q->n + 7) / 8) != 0) ++bad_count;
      free(bad);
    }
  }
  return (void*)bad_count;
}

static int unhex(const char* s, unsigned char* out, size_t n) {
  if (strlen(s) != 2 * n) return -1;
  for (size_t i = 0; i < n; ++i) {
    unsigned v;
    if (sscanf(s + 2 * i, "%2x", &v) != 1) return -1;
    out[i] = (unsigned char)v;
  }
  return 0;
}

static void puthex(const unsigned char* p, size_t n) {
  for (size_t i = 0; i < n; ++i) printf("%02x", p[i]);
}

int main(void) {
  int rc = nwc_init(1);
  if (rc != NWC_OK) {
    printf("INIT %d %s\n", rc, nwc_last_error());
    return 2;
  }
  static char line[1 << 20];
  while (fgets(line, sizeof line, stdin)) {
    char* tok = strtok(line, " \n");
    if (!tok) continue;
    if (tok[0] == 'S') {
      unsigned char m[32], pk[32], sig[64];
      const char* a = strtok(NULL, " \n");
      const char* b = strtok(NULL, " \n");
      const char* c = strtok(NULL, " \n");
      if (!a || !b || !c || unhex(a, m, 32) || unhex(b, pk, 32) || unhex(c, sig, 64)) return 3;
      printf("S %d\n", nwc_verify_strict(m, pk, sig));
    } else if (tok[0] == 'B') {
      unsigned char m[32];
      const char* a = strtok(NULL, " \n");
      const char* cnt = strtok(NULL, " \n");
      if (!a || !cnt || unhex(a, m, 32)) return 3;
      const size_t n = (size_t)strtoul(cnt, NULL, 10);
      unsigned char* pks = malloc(32 * n + 1);
      unsigned char* sigs = malloc(64 * n + 1);
      unsigned char* bad = calloc(n / 8 + 1, 1);
      for (size_t i = 0; i < n; ++i) {
        const char* p = strtok(NULL, " \n");
        const char* s = strtok(NULL, " \n");
        if (!p || !s || unhex(p, pks + 32 * i, 32) || unhex(s, sigs + 64 * i, 64)) return 3;
      }
      rc = nwc_verify_batch(m, pks, sigs, n, bad);
      printf("B %d ", rc);
      puthex(bad, (n + 7) / 8);
      printf("\n");
      if (g_nb < sizeof g_b / sizeof g_b[0]) {
        breq* q = &g_b[g_nb++];
        memcpy(q->m, m, 32);
        q->pks = pks;
        q->sigs = sigs;
        q->n = n;
        q->rc = rc;
        q->bad = bad;
      } else {
        free(pks);
        free(sigs);
        free(bad);
      }
    } else if (tok[0] == 'V') {
      const char* cnt = strtok(NULL, " \n");
      if (!cnt) return 3;
      const size_t n = (size_t)strtoul(cnt, NULL, 10);
      unsigned char* ms = malloc(32 * n + 1);
      unsigned char* pks = malloc(32 * n + 1);
      unsigned char* sigs = malloc(64 * n + 1);
      unsigned char* bits = calloc(n / 8 + 1, 1);
      for (size_t i = 0; i < n; ++i) {
        if (!fgets(line, sizeof line, stdin)) return 3;
        const char* a = strtok(line, " \n");
        const char* b = strtok(NULL, " \n");
        const char* c = strtok(NULL, " \n");
        if (!a || !b || !c || unhex(a, ms + 32 * i, 32) || unhex(b, pks + 32 * i, 32) || unhex(c, sigs + 64 * i, 64))
          return 3;
      }
      rc = nwc_verify_strict_many(ms, pks, sigs, n, bits);
      printf("V %d ", rc);
      puthex(bits, (n + 7) / 8);
      printf("\n");
      free(ms);
      free(pks);
      free(sigs);
      free(bits);
    } else if (tok[0] == 'C') {
      const char* cnt = strtok(NULL, " \n");
      if (!cnt) return 3;
      const size_t mc = (size_t)strtoul(cnt, NULL, 10);
      uint32_t* offs = malloc(4 * (mc + 1));
      for (size_t c = 0; c <= mc; ++c) {
        const char* o = strtok(NULL, " \n");
        if (!o) return 3;
        offs[c] = (uint32_t)strtoul(o, NULL, 10);
      }
      const size_t nv = offs[mc];
      unsigned char* pks = malloc(32 * nv + 1);
      unsigned char* sigs = malloc(64 * nv + 1);
      unsigned char* dig = malloc(32 * mc + 1);
      for (size_t i = 0; i < nv; ++i) {
        if (!fgets(line, sizeof line, stdin)) return 3;
        const char* b = strtok(line, " \n");
        const char* c = strtok(NULL, " \n");
        if (!b || !c || unhex(b, pks + 32 * i, 32) || unhex(c, sigs + 64 * i, 64)) return 3;
      }
      for (size_t c = 0; c < mc; ++c) {
        if (!fgets(line, sizeof line, stdin)) return 3;
        const char* a = strtok(line, " \n");
        if (!a || unhex(a, dig + 32 * c, 32)) return 3;
      }
      unsigned char* cert = calloc(mc / 8 + 1, 1);
      unsigned char* badv = calloc(nv / 8 + 1, 1);
      rc = nwc_verify_batch_many(dig, offs, pks, sigs, mc, cert, badv);
      printf("C %d ", rc);
      puthex(cert, (mc + 7) / 8);
      printf(" ");
      puthex(badv, (nv + 7) / 8);
      printf("\n");
      free(offs);
      free(pks);
      free(sigs);
      free(dig);
      free(cert);
      free(badv);
    } else if (tok[0] == 'X') {
      const char* t = strtok(NULL, " \n");
      const char* r = strtok(NULL, " \n");
      if (!t || !r) return 3;
      const int threads = atoi(t);
      g_rounds = atoi(r);
      pthread_t th[64];
      long mism = 0;
      for (int k = 0; k < threads && k < 64; ++k) pthread_create(&th[k], NULL, worker, NULL);
      for (int k = 0; k < threads && k < 64; ++k) {
        void* v = NULL;
        pthread_join(th[k], &v);
        mism += (long)v;
      }
      printf("X %ld\n", mism);
    } else if (tok[0] == 'K') {
      /* K n pk... : nwc_set_committee (n = 0 clears it) */
      const char* cnt = strtok(NULL, " \n");
      if (!cnt) return 3;
      const size_t n = (size_t)strtoul(cnt, NULL, 10);
      unsigned char* pks = malloc(32 * n + 1);
      for (size_t i = 0; i < n; ++i) {
        const char* p = strtok(NULL, " \n");
        if (!p || unhex(p, pks + 32 * i, 32)) return 3;
      }
      printf("K %d\n", nwc_set_committee(n ? pks : NULL, n));
      free(pks);
    } else if (tok[0] == 'L') {
      /* L calls warm msg n pk sig ... : per-call latency of nwc_verify_batch on one batch, timed
       * here in C (no interpreter in the loop); prints the first two calls and percentiles of
       * calls warm.. in microseconds */
      const char* c1 = strtok(NULL, " \n");
      const char* c2 = strtok(NULL, " \n");
      const char* a = strtok(NULL, " \n");
      const char* cnt = strtok(NULL, " \n");
      unsigned char m[32];
      if (!c1 || !c2 || !a || !cnt || unhex(a, m, 32)) return 3;
      const long calls = atol(c1), warm = atol(c2);
      const size_t n = (size_t)strtoul(cnt, NULL, 10);
      unsigned char* pks = malloc(32 * n + 1);
      unsigned char* sigs = malloc(64 * n + 1);
      for (size_t i = 0; i < n; ++i) {
        const char* p = strtok(NULL, " \n");
        const char* s = strtok(NULL, " \n");
        if (!p || !s || unhex(p, pks + 32 * i, 32) || unhex(s, sigs + 64 * i, 64)) return 3;
      }
      double* us = malloc(sizeof(double) * (size_t)(calls + 1));
      int rc0 = -100;
      for (long k = 0; k < calls; ++k) {
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        rc = nwc_verify_batch(m, pks, sigs, n, NULL);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if (k == 0) rc0 = rc;
        if (rc != rc0) return 4;
        us[k] = (t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_nsec - t0.tv_nsec) * 1e-3;
      }
      const double first = us[0], second = calls > 1 ? us[1] : 0;
      const long cnt2 = calls - warm;
      double* w = us + warm;
      qsort(w, (size_t)cnt2, sizeof(double), cmp_double);
      double sum = 0;
      for (long k = 0; k < cnt2; ++k) sum += w[k];
      printf("L %d %.2f %.2f %.2f %.2f %.2f %.2f %.2f %.2f\n", rc0, first, second, w[cnt2 / 2], w[(long)(cnt2 * 0.9)],
             w[(long)(cnt2 * 0.99)], w[(long)(cnt2 * 0.999)], w[cnt2 - 1], sum / cnt2);
      free(us);
      free(pks);
      free(sigs);
    } else if (tok[0] == 'Z') {
      /* sanitizer self-check (tests only): one byte read past a heap block must be reported */
      volatile unsigned char* z = malloc(16);
      printf("Z %d\n", z[16]);
      free((void*)z);
    } else if (tok[0] == 'D') {
      const char* a = strtok(NULL, " \n");
      const size_t len = a ? strlen(a) / 2 : 0;
      unsigned char* data = malloc(len + 1);
      if (len && unhex(a, data, len)) return 3;
      uint64_t offs[2] = {0, len};
      unsigned char out[32];
      rc = nwc_sha512_trunc32_many(data, offs, 1, out);
      if (rc) {
        printf("D ERR %d\n", rc);
      } else {
        printf("D ");
        puthex(out, 32);
        printf("\n");
      }
      free(data);
    }
    fflush(stdout);
  }
  for (size_t i = 0; i < g_nb; ++i) {
    free(g_b[i].pks);
    free(g_b[i].sigs);
    free(g_b[i].bad);
  }
  nwc_shutdown();
  return 0;
}
