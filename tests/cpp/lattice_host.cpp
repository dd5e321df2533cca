// Host build of narwhal_amd/csrc/lattice.h (the same source the kernels use) for CPU tests.
#include "lattice.h"
template <bool LEHMER>
static void run(const uint32_t k[8], uint32_t c[5], uint32_t d[5], int* c_neg, int* ok) {
  nwc::lat::HalfScalars h = nwc::lat::reduce<LEHMER>(k);
  for (int i = 0; i < 5; ++i) { c[i] = h.c[i]; d[i] = h.d[i]; }
  *c_neg = h.c_neg;
  *ok = h.ok;
}
// the kernels' reduction (Lehmer blocks)
extern "C" void lat_reduce(const uint32_t k[8], uint32_t c[5], uint32_t d[5], int* c_neg, int* ok) {
  run<true>(k, c, d, c_neg, ok);
}
// one exact step at a time: the same remainder sequence, so the same (c, d)
extern "C" void lat_reduce_single(const uint32_t k[8], uint32_t c[5], uint32_t d[5], int* c_neg, int* ok) {
  run<false>(k, c, d, c_neg, ok);
}
