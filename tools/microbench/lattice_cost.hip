// Development microbenchmark: device cost of lat::reduce (half-size scalars) per lane, against a
// SHA-512 block, on 1M pseudo-random k.  hipcc --offload-arch=gfx950 -O3 -I narwhal_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "lattice.h"
#include "sha512.h"
using namespace nwc;

template <bool LEHMER>
__global__ __launch_bounds__(256, 2) void k_lat(const uint32_t* ks, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  for (int j = 0; j < 8; ++j) k[j] = ks[8 * i + j];
  k[7] &= 0x0FFFFFFFu;
  lat::HalfScalars h = lat::reduce<LEHMER>(k);
  out[i] = h.c[0] ^ h.d[1] ^ (h.ok ? 1u : 0u) ^ (uint32_t)h.bits;
}
__global__ __launch_bounds__(256, 2) void k_sha(const uint32_t* ks, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t w[16], st[8];
  for (int j = 0; j < 16; ++j) w[j] = ((uint64_t)ks[8 * i + (j & 7)] << 32) | j;
  sha512_init_state(st);
  sha512_compress(st, w);
  out[i] = (uint32_t)st[0] ^ (uint32_t)st[3];
}
int main() {
  const int n = 1 << 20;
  std::vector<uint32_t> h(8 * (size_t)n);
  uint64_t x = 88172645463325252ull;
  for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x; }
  uint32_t *dk, *dout;
  hipMalloc(&dk, 32 * (size_t)n);
  hipMalloc(&dout, 4 * (size_t)n);
  hipMemcpy(dk, h.data(), 32 * (size_t)n, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int kind = 0; kind < 3; ++kind) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (kind == 0) k_lat<true><<<n / 256, 256>>>(dk, dout, n);
      else if (kind == 1) k_lat<false><<<n / 256, 256>>>(dk, dout, n);
      else k_sha<<<n / 256, 256>>>(dk, dout, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep == 2) printf("%s: %.3f ms per 1M lanes\n", kind == 2 ? "sha512 block" : kind == 1 ? "lat::reduce<single steps>" : "lat::reduce<Lehmer>", ms);
    }
  }
  return 0;
}
