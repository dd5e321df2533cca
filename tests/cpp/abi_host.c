/* A plain C host of libnwc.so -- what the Rust `crypto` shim does, with no
 * Python or torch in the process: init, Signature::verify, Signature::verify_batch with its
 * bad-vote bitmap, and the worker's batch digest.
 *
 * stdin, one request per line (hex fields):
 *   S <msg32> <pk32> <sig64>            -> "S <rc>"                 (nwc_verify_strict)
 *   B <msg32> <n> <pk32 sig64> x n      -> "B <rc> <bad bitmap>"    (nwc_verify_batch)
 *   D <data>                            -> "D <digest32>"           (nwc_sha512_trunc32_many)
 * Built by __graft_entry__.build() into tests/cpp/build/abi_host; run by tests/test_gpu_abi_host.py.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nwc.h"

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
      free(pks);
      free(sigs);
      free(bad);
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
  nwc_shutdown();
  return 0;
}
