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
 *   T <m> <offsets m+1>, votes and digests as C -> "T <rc> <cert bitmap> <bad bitmap>"
 *                                          (nwc_verify_batch_straus_many)
 *   P <m> ..., as T                          -> "P <rc> ..."  (nwc_verify_batch_msm_many)
 *   Q <n>, then n lines <pk32 stake nworkers wid...>  -> "Q <rc>"  (nwc_set_committee_config)
 *   M <m> <gc_round> <target72 | ->, then m lines <msg hex> -> "M <rc> <code,kind,digest32>..."
 *                                          (nwc_sanitize_messages)
 *   G <max_group> <wait_us> <arena 0/1> <n>, then n lines <data hex | ->
 *                                       -> per result "g <tag> <digest32>" or "g <tag> ERR <rc>",
 *                                          then "G <destroy rc>": a digester fed every batch (from
 *                                          malloc'd buffers, or written into its receive arena),
 *                                          polled until every tag is back; the batches and their
 *                                          digests are kept for Y
 *   W <k>                               -> "W <mismatches>": the last V request tiled k times through
 *                                          nwc_verify_strict_many (large enough for the pipelined
 *                                          chunks and the pinned host stages), bits vs V's
 *   Y <verify threads> <rounds>         -> "Y <mismatches>": one thread streams the last G's
 *                                          batches through a new digester `rounds` times while
 *                                          the verify threads re-run every B request and the
 *                                          last V request on the same device
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
#include <unistd.h>

#include "nwc.h"

#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#define NWC_HOST_ASAN 1
#include <sanitizer/lsan_interface.h>
#endif
#endif

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
/* the last V request (re-run by Y) */
static unsigned char *g_vm, *g_vp, *g_vs, *g_vbits;
static size_t g_vn;
/* the last G command's batches and digests (streamed again by Y) */
static unsigned char** g_gb;
static size_t* g_glen;
static unsigned char* g_gdig;
static size_t g_gn;

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

/* Y: one digester streaming the G batches `g_rounds` times, compared with the G digests */
static void* digest_streamer(void* arg) {
  long mism = 0;
  (void)arg;
  nwc_digester* q = nwc_digester_create(64, 500);
  if (!q) return (void*)1000000L;
  uint64_t* tags = malloc(sizeof(uint64_t) * (g_gn + 1));
  unsigned char* dig = malloc(32 * (g_gn + 1));
  for (int r = 0; r < g_rounds; ++r) {
    for (size_t i = 0; i < g_gn; ++i)
      if (nwc_digester_submit(q, g_gb[i], g_glen[i], (uint64_t)r * g_gn + i) != 0) ++mism;
    size_t got = 0;
    while (got < g_gn) {
      size_t n = 0;
      if (nwc_digester_poll(q, g_gn - got, 200000, tags, dig, &n) != 0) { ++mism; break; }
      for (size_t k = 0; k < n; ++k) {
        const uint64_t want = (uint64_t)r * g_gn + got + k;
        if (tags[k] != want || memcmp(dig + 32 * k, g_gdig + 32 * (want - (uint64_t)r * g_gn), 32) != 0) ++mism;
      }
      got += n;
    }
  }
  if (nwc_digester_destroy(q) != 0) ++mism;
  free(tags);
  free(dig);
  return (void*)mism;
}

/* Y: the B requests and the last V request, re-run */
static void* verifier(void* arg) {
  long mism = (long)(size_t)worker(arg);
  for (int r = 0; r < g_rounds && g_vn; ++r) {
    unsigned char* bits = calloc(g_vn / 8 + 1, 1);
    if (nwc_verify_strict_many(g_vm, g_vp, g_vs, g_vn, bits) != 0 || memcmp(bits, g_vbits, (g_vn + 7) / 8) != 0)
      ++mism;
    free(bits);
  }
  return (void*)mism;
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
      free(g_vm);
      free(g_vp);
      free(g_vs);
      free(g_vbits);
      g_vm = ms;
      g_vp = pks;
      g_vs = sigs;
      g_vbits = bits;
      g_vn = rc == 0 ? n : 0;
    } else if (tok[0] == 'C' || tok[0] == 'T' || tok[0] == 'P') {
      const char kind = tok[0];
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
      rc = kind == 'C'   ? nwc_verify_batch_many(dig, offs, pks, sigs, mc, cert, badv)
           : kind == 'T' ? nwc_verify_batch_straus_many(dig, offs, pks, sigs, mc, cert, badv)
                         : nwc_verify_batch_msm_many(dig, offs, pks, sigs, mc, cert, badv);
      printf("%c %d ", kind, rc);
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
    } else if (tok[0] == 'Q') {
      /* Q n, then n lines "pk stake nworkers wid...": nwc_set_committee_config */
      const char* cnt = strtok(NULL, " \n");
      if (!cnt) return 3;
      const size_t n = (size_t)strtoul(cnt, NULL, 10);
      unsigned char* pks = malloc(32 * n + 1);
      uint64_t* stakes = malloc(8 * n + 8);
      uint32_t* woff = malloc(4 * (n + 1));
      uint32_t* wids = malloc(4 * (8 * n + 1));
      woff[0] = 0;
      for (size_t i = 0; i < n; ++i) {
        if (!fgets(line, sizeof line, stdin)) return 3;
        const char* p = strtok(line, " \n");
        const char* st = strtok(NULL, " \n");
        const char* nw = strtok(NULL, " \n");
        if (!p || !st || !nw || unhex(p, pks + 32 * i, 32)) return 3;
        stakes[i] = strtoull(st, NULL, 10);
        const unsigned k = (unsigned)strtoul(nw, NULL, 10);
        if (k > 8) return 3;
        woff[i + 1] = woff[i] + k;
        for (unsigned j = 0; j < k; ++j) {
          const char* w = strtok(NULL, " \n");
          if (!w) return 3;
          wids[woff[i] + j] = (uint32_t)strtoul(w, NULL, 10);
        }
      }
      printf("Q %d\n", nwc_set_committee_config(pks, stakes, n, woff, wids));
      free(pks);
      free(stakes);
      free(woff);
      free(wids);
    } else if (tok[0] == 'M') {
      /* M m gc_round target|-, then m message lines: nwc_sanitize_messages */
      const char* cnt = strtok(NULL, " \n");
      const char* gc = strtok(NULL, " \n");
      const char* tg = strtok(NULL, " \n");
      if (!cnt || !gc || !tg) return 3;
      const size_t m = (size_t)strtoul(cnt, NULL, 10);
      const uint64_t gc_round = strtoull(gc, NULL, 10);   /* before the message lines overwrite `line` */
      unsigned char target[72];
      const int has_target = strcmp(tg, "-") != 0;
      if (has_target && unhex(tg, target, 72)) return 3;
      unsigned char** msg = malloc(sizeof(unsigned char*) * (m + 1));
      size_t* len = malloc(sizeof(size_t) * (m + 1));
      size_t total = 0;
      for (size_t i = 0; i < m; ++i) {
        if (!fgets(line, sizeof line, stdin)) return 3;
        const char* h = strtok(line, " \n");
        len[i] = (h && strcmp(h, "-") != 0) ? strlen(h) / 2 : 0;
        msg[i] = malloc(len[i] + 1);
        if (len[i] && unhex(h, msg[i], len[i])) return 3;
        total += len[i];
      }
      unsigned char* data = malloc(total + 1);
      uint64_t* offs = malloc(8 * (m + 1));
      offs[0] = 0;
      for (size_t i = 0; i < m; ++i) {
        memcpy(data + offs[i], msg[i], len[i]);
        offs[i + 1] = offs[i] + len[i];
        free(msg[i]);
      }
      int32_t* codes = malloc(4 * (m + 1));
      unsigned char* digs = malloc(32 * (m + 1));
      unsigned char* kinds = malloc(m + 1);
      rc = nwc_sanitize_messages(data, offs, m, gc_round, has_target ? target : NULL, codes, digs, kinds);
      printf("M %d", rc);
      for (size_t i = 0; rc == 0 && i < m; ++i) {
        printf(" %d,%d,", codes[i], kinds[i]);
        puthex(digs + 32 * i, 32);
      }
      printf("\n");
      free(msg);
      free(len);
      free(data);
      free(offs);
      free(codes);
      free(digs);
      free(kinds);
    } else if (tok[0] == 'G') {
      /* G max_group wait_us arena n, then n data lines: the worker digester end to end */
      const char* a1 = strtok(NULL, " \n");
      const char* a2 = strtok(NULL, " \n");
      const char* a3 = strtok(NULL, " \n");
      const char* a4 = strtok(NULL, " \n");
      if (!a1 || !a2 || !a3 || !a4) return 3;
      const uint32_t max_group = (uint32_t)strtoul(a1, NULL, 10), wait_us = (uint32_t)strtoul(a2, NULL, 10);
      const int use_arena = atoi(a3);
      const size_t n = (size_t)strtoul(a4, NULL, 10);
      for (size_t i = 0; i < g_gn; ++i) free(g_gb[i]);
      free(g_gb);
      free(g_glen);
      free(g_gdig);
      g_gb = malloc(sizeof(unsigned char*) * (n + 1));
      g_glen = malloc(sizeof(size_t) * (n + 1));
      g_gdig = calloc(32 * (n + 1), 1);
      g_gn = n;
      size_t arena_bytes = 16;
      for (size_t i = 0; i < n; ++i) {
        if (!fgets(line, sizeof line, stdin)) return 3;
        const char* h = strtok(line, " \n");
        g_glen[i] = (h && strcmp(h, "-") != 0) ? strlen(h) / 2 : 0;
        g_gb[i] = malloc(g_glen[i] + 1);
        if (g_glen[i] && unhex(h, g_gb[i], g_glen[i])) return 3;
        arena_bytes += (g_glen[i] + 15) & ~(size_t)15;
      }
      nwc_digester* q = nwc_digester_create(max_group, wait_us);
      if (!q) {
        printf("G CREATE %s\n", nwc_last_error());
        fflush(stdout);
        continue;
      }
      unsigned char* arena = use_arena ? nwc_digester_arena(q, arena_bytes) : NULL;
      if (use_arena && !arena) return 5;
      size_t off = 0;
      size_t submitted = 0;
      for (size_t i = 0; i < n; ++i) {
        const unsigned char* src = g_gb[i];
        if (arena) {   /* received straight into the arena, at 16-byte-rounded offsets */
          memcpy(arena + off, g_gb[i], g_glen[i]);
          src = arena + off;
          off += (g_glen[i] + 15) & ~(size_t)15;
        }
        rc = nwc_digester_submit(q, src, g_glen[i], i);
        if (rc != 0) {
          printf("g %zu SUBMIT %d\n", i, rc);
          continue;
        }
        ++submitted;
      }
      uint64_t* tags = malloc(sizeof(uint64_t) * (n + 1));
      unsigned char* dig = malloc(32 * (n + 1));
      size_t back = 0;
      int idle = 0;
      while (back < submitted && idle < 50) {
        size_t k = 0;
        rc = nwc_digester_poll(q, n, 100000, tags, dig, &k);
        idle = k ? 0 : idle + 1;
        for (size_t j = 0; j < k; ++j) {
          if (rc == 0) {
            printf("g %llu ", (unsigned long long)tags[j]);
            puthex(dig + 32 * j, 32);
            printf("\n");
            memcpy(g_gdig + 32 * tags[j], dig + 32 * j, 32);
          } else {
            printf("g %llu ERR %d\n", (unsigned long long)tags[j], rc);
          }
        }
        back += k;
        if (rc != 0 && k == 0) break;   /* sticky error, nothing left */
      }
      free(tags);
      free(dig);
      printf("G %d\n", nwc_digester_destroy(q));
    } else if (tok[0] == 'W') {
      const char* t = strtok(NULL, " \n");
      if (!t || !g_vn) return 3;
      const size_t k = (size_t)strtoul(t, NULL, 10), n = g_vn * k;
      unsigned char* ms = malloc(32 * n + 1);
      unsigned char* ps = malloc(32 * n + 1);
      unsigned char* ss = malloc(64 * n + 1);
      unsigned char* bits = calloc(n / 8 + 1, 1);
      for (size_t j = 0; j < k; ++j) {
        memcpy(ms + 32 * g_vn * j, g_vm, 32 * g_vn);
        memcpy(ps + 32 * g_vn * j, g_vp, 32 * g_vn);
        memcpy(ss + 64 * g_vn * j, g_vs, 64 * g_vn);
      }
      long mism = nwc_verify_strict_many(ms, ps, ss, n, bits) != 0 ? 1000000 : 0;
      for (size_t i = 0; i < n; ++i) {
        const size_t v = i % g_vn;
        mism += ((bits[i >> 3] >> (i & 7)) & 1) != ((g_vbits[v >> 3] >> (v & 7)) & 1);
      }
      printf("W %ld\n", mism);
      free(ms);
      free(ps);
      free(ss);
      free(bits);
    } else if (tok[0] == 'Y') {
      const char* t = strtok(NULL, " \n");
      const char* r = strtok(NULL, " \n");
      if (!t || !r) return 3;
      const int threads = atoi(t);
      g_rounds = atoi(r);
      pthread_t th[65];
      long mism = 0;
      int k = 0;
      pthread_create(&th[k++], NULL, digest_streamer, NULL);
      for (int j = 0; j < threads && k < 65; ++j) pthread_create(&th[k++], NULL, verifier, NULL);
      for (int j = 0; j < k; ++j) {
        void* v = NULL;
        pthread_join(th[j], &v);
        mism += (long)v;
      }
      printf("Y %ld\n", mism);
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
  for (size_t i = 0; i < g_gn; ++i) free(g_gb[i]);
  free(g_gb);
  free(g_glen);
  free(g_gdig);
  free(g_vm);
  free(g_vp);
  free(g_vs);
  free(g_vbits);
  nwc_shutdown();
  fflush(stdout);
#ifdef NWC_HOST_ASAN
  /* Leak check of everything the process still holds once the library is shut down (the
   * sanitized build runs with detect_leaks=1; the suppressions name libhsa-runtime64 and
   * libamdhip64 frames only, tests/cpp/lsan.supp): a libnwc allocation still reachable from
   * nowhere is reported with its stack and fails the run. */
  if (__lsan_do_recoverable_leak_check()) {
    fprintf(stderr, "abi_host: leaks after nwc_shutdown\n");
    fflush(stderr);
    _exit(5);
  }
#endif
  /* NWC_HOST_EXIT=return: leave through main's return, i.e. exit() with the atexit handlers,
   * libnwc's static destructors and the HIP/HSA runtime's own teardown.  Under ASan with its
   * default quarantine that teardown aborts: an operator delete inside libamdhip64's
   * __cxa_finalize (libhsa-runtime64 frames) pushes the quarantine over its limit, the recycle
   * frees an older quarantined device-allocator chunk, and ASan's device allocator CHECKs
   * "dev_runtime_unloaded_" -- no libnwc frame is involved, and with quarantine_size_mb=0 the
   * same exit is clean (profiles/r05/asan_exit.md; the test runs it that way).  By default the
   * host leaves with _exit: libnwc's own teardown (nwc_shutdown, above) and the leak check have
   * run under the sanitizers by then, with the quarantine on for use-after-free detection. */
  const char* how = getenv("NWC_HOST_EXIT");
  if (how && strcmp(how, "return") == 0) return 0;
  fflush(stderr);
  _exit(0);
}
