// Limb-sliced point operations (ge_sliced.h) against the one-point-per-lane ones (ge25519.h):
// every wave builds its own point P_w (per-lane code), then compares gs_dbl / gs_to_p2 / gs_to_p3
// / gs_add_cached and the torsion test l*P against ge_p2_dbl / ge_p1p1_to_* / ge_add_cached /
// ge_has_torsion (canonical encodings of the affine results), for P_w and P_w + T2 (T2 = (0, -1),
// of order 2: l (P + T2) = T2, so the sliced test must report torsion there and none for P_w).
// Prints mismatch counts and the latency of one torsion test both ways (one wave on the GPU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "fe25519.h"
#include "consts.h"
#include "ge25519.h"
#include "sc25519.h"
#include "ge_sliced.h"
using namespace nwc;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ ge_p3 base_point() {
  ge_p3 b;
  b.X = FE_BASE_X; b.Y = FE_BASE_Y; b.Z = fe_one(); b.T = fe_mul(FE_BASE_X, FE_BASE_Y);
  return b;
}
// kernels.hip's ge_has_torsion, restated here (one point per lane)
__device__ __noinline__ bool ge_has_torsion(const ge_p3& P) {
  const ge_cached pc = ge_p3_to_cached(P);
  ge_p2 acc = ge_p3_to_p2(P);
  for (int bit = 251; bit >= 0; --bit) {
    ge_p1p1 t = ge_p2_dbl(acc);
    if ((SC_L[bit >> 5] >> (bit & 31)) & 1u) t = ge_add_cached(ge_p1p1_to_p3(t), pc);
    acc = ge_p1p1_to_p2(t);
  }
  return !(fe_is_zero(acc.X) && fe_is_zero(fe_sub(acc.Y, acc.Z)));
}
// affine canonical (x, y) words of a projective point (one inversion, test only)
__device__ void affine_words(const fe& X, const fe& Y, const fe& Z, u32 out[16]) {
  fe t = fe_sqn(fe_pow22523(Z), 3);
  const fe zi = fe_mul(t, fe_mul(fe_sq(Z), Z));
  fe_to_words(fe_mul(X, zi), out);
  fe_to_words(fe_mul(Y, zi), out + 8);
}
__device__ gs_p3 to_gs(const ge_p3& p) { return {fes_from_fe(p.X), fes_from_fe(p.Y), fes_from_fe(p.Z), fes_from_fe(p.T)}; }

// out per wave: [0] dbl mismatch, [1] add mismatch, [2] torsion(P) sliced, [3] torsion(P) lane,
// [4] torsion(P+T2) sliced, [5] torsion(P+T2) lane
__global__ void k_check(unsigned* out) {
  const int w = blockIdx.x;
  ge_p3 P = base_point();
  const ge_cached bc = ge_p3_to_cached(P);
  for (int k = 0; k < 3 + (w % 7); ++k) P = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(P)));
  for (int k = 0; k < 1 + w; ++k) P = ge_p1p1_to_p3(ge_add_cached(P, bc));
  // lane reference
  const ge_p1p1 d1 = ge_p2_dbl(ge_p3_to_p2(P));
  const ge_p2 d2 = ge_p1p1_to_p2(d1);
  const ge_p3 a3 = ge_p1p1_to_p3(ge_add_cached(ge_p1p1_to_p3(d1), bc));
  // sliced
  const gs_p3 S = to_gs(P);
  const gs_p1p1 sd1 = gs_dbl(gs_p3_to_p2(S));
  const gs_p2 sd2 = gs_to_p2(sd1);
  const gs_cached sbc = gs_to_cached(to_gs(base_point()));
  const gs_p3 sa3 = gs_to_p3(gs_add_cached(gs_to_p3(sd1), sbc));
  u32 e1[16], e2[16], e3[16], e4[16];
  affine_words(d2.X, d2.Y, d2.Z, e1);
  affine_words(fe_from_fes(sd2.X), fe_from_fes(sd2.Y), fe_from_fes(sd2.Z), e2);
  affine_words(a3.X, a3.Y, a3.Z, e3);
  affine_words(fe_from_fes(sa3.X), fe_from_fes(sa3.Y), fe_from_fes(sa3.Z), e4);
  unsigned m1 = 0, m2 = 0;
  for (int i = 0; i < 16; ++i) { m1 |= e1[i] ^ e2[i]; m2 |= e3[i] ^ e4[i]; }
  // torsion: P and P + T2 (T2 = (0, -1): negate X and Y of an extended point)
  ge_p3 PT = P;
  PT.X = fe_neg(P.X); PT.Y = fe_neg(P.Y);
  const bool ts = gs_has_torsion(to_gs(P), SC_L), tl = ge_has_torsion(P);
  const bool tts = gs_has_torsion(to_gs(PT), SC_L), ttl = ge_has_torsion(PT);
  if (threadIdx.x == 0) {
    out[6 * w + 0] = m1 != 0; out[6 * w + 1] = m2 != 0;
    out[6 * w + 2] = ts; out[6 * w + 3] = tl; out[6 * w + 4] = tts; out[6 * w + 5] = ttl;
  }
}

// x-only chain (gs_xonly_dbl_n) vs Edwards doublings: u([2^k] P) == (Z + Y) / (Z - Y) of the
// per-lane [2^k] P, for k = 1, 7 and 252, cross-multiplied; out[w] = number of mismatches
__global__ void k_xonly_check(unsigned* out) {
  const int w = blockIdx.x;
  ge_p3 P = base_point();
  const ge_cached bc = ge_p3_to_cached(P);
  for (int k = 0; k < 1 + w; ++k) P = ge_p1p1_to_p3(ge_add_cached(P, bc));
  if (w & 1) { P.X = fe_neg(P.X); P.Y = fe_neg(P.Y); }   // odd waves: P + T2 (a torsion component)
  // affine y of P
  u32 aw[16];
  affine_words(P.X, P.Y, P.Z, aw);
  const fe y = fe_tighten(fe_from_words(aw + 8));   // as in k_verify_cold (fes_mul input bounds)
  unsigned bad = 0;
  const int ks[3] = {1, 7, 252};
  for (int j = 0; j < 3; ++j) {
    fes U, W;
    gs_xonly_dbl_n(fes_from_fe(y), ks[j], U, W);
    ge_p2 q = ge_p3_to_p2(P);
    for (int k = 0; k < ks[j]; ++k) q = ge_p1p1_to_p2(ge_p2_dbl(q));
    const fe lhs = fe_mul(fe_from_fes(U), fe_sub(q.Z, q.Y));
    const fe rhs = fe_mul(fe_from_fes(W), fe_add(q.Z, q.Y));
    bad += fe_is_zero(fe_sub(lhs, rhs)) ? 0u : 1u;
  }
  if (threadIdx.x == 0) out[w] = bad;
}

__global__ void k_tors_lane(const ge_p3* P, unsigned* out) {
  if (threadIdx.x == 0) out[0] = ge_has_torsion(P[0]);
}
__global__ void k_tors_sliced(const ge_p3* P, unsigned* out) {
  const bool t = gs_has_torsion(to_gs(P[0]), SC_L);
  if (threadIdx.x == 0) out[0] = t;
}
__global__ void k_one_point(ge_p3* P) {
  if (threadIdx.x == 0) { ge_p3 p = base_point(); p = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(p))); P[0] = p; }
}

int main() {
  const int W = 64;
  unsigned* d;
  CHECK(hipMalloc(&d, 6 * W * sizeof(unsigned)));
  hipLaunchKernelGGL(k_check, dim3(W), dim3(64), 0, 0, d);
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned> h(6 * W);
  CHECK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
  int bad_dbl = 0, bad_add = 0, bad_tors = 0;
  for (int w = 0; w < W; ++w) {
    bad_dbl += h[6 * w];
    bad_add += h[6 * w + 1];
    bad_tors += (h[6 * w + 2] != 0) + (h[6 * w + 3] != 0) + (h[6 * w + 4] != 1) + (h[6 * w + 5] != 1);
  }
  printf("points %d: dbl mismatches %d, add mismatches %d, torsion-test errors %d\n", W, bad_dbl, bad_add, bad_tors);
  hipLaunchKernelGGL(k_xonly_check, dim3(W), dim3(64), 0, 0, d);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h.data(), d, W * 4, hipMemcpyDeviceToHost));
  int bad_x = 0;
  for (int w = 0; w < W; ++w) bad_x += h[w];
  printf("x-only u([2^k] P) vs Edwards doublings (k = 1, 7, 252; half the points with torsion): %d mismatches of %d\n",
         bad_x, 3 * W);
  bad_tors += bad_x;
  ge_p3* P;
  CHECK(hipMalloc(&P, sizeof(ge_p3)));
  hipLaunchKernelGGL(k_one_point, dim3(1), dim3(64), 0, 0, P);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    float ms_l = 0, ms_s = 0;
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_tors_lane, dim3(1), dim3(64), 0, 0, P, d);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms_l, e0, e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_tors_sliced, dim3(1), dim3(64), 0, 0, P, d);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms_s, e0, e1));
    printf("torsion test of one key: one lane %.1f us, limb-sliced wave %.1f us\n", ms_l * 1e3, ms_s * 1e3);
  }
  return (bad_dbl || bad_add || bad_tors) ? 2 : 0;
}
