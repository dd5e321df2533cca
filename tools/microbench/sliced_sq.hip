// Latency of one dependent chain of field squarings in ONE wave (the critical path of the
// latency kernel's square root): fe_sq with one element per lane vs fes_sq with one element per
// 16-lane row (fe_sliced.h).  Also checks that both chains give the same canonical result, and
// times z^(2^252-3) both ways.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "fe25519.h"
#include "consts.h"
#include "fe_sliced.h"
using namespace nwc;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ fe seed_fe(unsigned s) {
  fe a;
  for (int i = 0; i < 10; ++i) a.v[i] = (i32)((s * 2654435761u + i * 40503u) & ((1u << ((i & 1) ? 24 : 25)) - 1u));
  return a;
}

__global__ void k_lane(int n, int pow, unsigned s, unsigned* out) {
  fe a = seed_fe(s);
  if (threadIdx.x == 0) {
    if (pow) { for (int r = 0; r < n; ++r) a = fe_pow22523(a); }
    else a = fe_sqn(a, n);
    u32 w[8];
    fe_to_words(a, w);
    for (int i = 0; i < 8; ++i) out[i] = w[i];
  }
}
__global__ void k_sliced(int n, int pow, unsigned s, unsigned* out) {
  fes a = fes_from_fe(seed_fe(s));
  if (pow) { for (int r = 0; r < n; ++r) a = fes_pow22523(a); }
  else a = fes_sqn(a, n);
  fe b = fe_from_fes(a);
  if (threadIdx.x == 0) {
    u32 w[8];
    fe_to_words(b, w);
    for (int i = 0; i < 8; ++i) out[i] = w[i];
  }
}

int main() {
  unsigned *d, h1[8], h2[8];
  CHECK(hipMalloc(&d, 64));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  int bad = 0;
  for (int pow = 0; pow < 2; ++pow) {
    const int n = pow ? 20 : 5000;
    float ms[2];
    for (int v = 0; v < 2; ++v) {
      for (int rep = 0; rep < 2; ++rep) {   // first launch warms up
        CHECK(hipEventRecord(e0));
        if (v == 0) hipLaunchKernelGGL(k_lane, dim3(1), dim3(64), 0, 0, n, pow, 12345u, d);
        else hipLaunchKernelGGL(k_sliced, dim3(1), dim3(64), 0, 0, n, pow, 12345u, d);
        CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms[v], e0, e1));
      }
      CHECK(hipMemcpy(v == 0 ? h1 : h2, d, 32, hipMemcpyDeviceToHost));
    }
    const bool same = memcmp(h1, h2, 32) == 0;
    bad |= !same;
    const double per = pow ? 1.0 : (double)n;
    printf("%s x%d: one lane %.3f us, sliced %.3f us per %s (%.2fx); results %s\n", pow ? "pow22523" : "squarings", n,
           ms[0] * 1e3 / (pow ? n : 1) / (pow ? 1 : 1), ms[1] * 1e3 / (pow ? n : 1), pow ? "exponentiation" : "chain",
           ms[0] / ms[1], same ? "equal" : "DIFFER");
    if (!pow) printf("  per squaring: one lane %.1f ns, sliced %.1f ns\n", ms[0] * 1e6 / per, ms[1] * 1e6 / per);
  }
  return bad;
}
