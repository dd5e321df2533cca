// 8 x 32-bit saturated field (tools/microbench/fe32.h) against the 10 x 25.5-bit one the kernels
// use (narwhal_amd/csrc/fe25519.h): equal results, and throughput at 1, 2 and 4 waves per SIMD.
//
//   fe32 [n_check] [iters]     writes /tmp/fe32_sub.bin (inputs and fe32 outputs of a subset, for
//                              tools/microbench/fe32_check.py) and prints one JSON line
//
// Check: n_check random pairs (uniform 256-bit, [p, 2^255), edge values) -- fe32 mul / sq / add /
// sub canonicalised vs fe_mul / fe_sq / fe_add / fe_sub + fe_to_words on the same value (bit 255
// cleared, which fe_from_words ignores), counted on the GPU; the subset file adds inputs with bit
// 255 set for the big-integer check.  Throughput: per lane two independent chains x <- x * y (or
// x <- x^2) for `iters` steps, 256-thread blocks, grid = waves per SIMD x CUs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "fe25519.h"
#include "fe32.h"

using nwc::fe;
using fe32x::fe32;
typedef uint32_t u32;
typedef uint64_t u64;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ fe32 ld32(const u32* p) { fe32 r; for (int i = 0; i < 8; ++i) r.v[i] = p[i]; return r; }
__device__ __forceinline__ fe ld10(const u32* p) {
  u32 w[8];
  for (int i = 0; i < 8; ++i) w[i] = p[i];
  return nwc::fe_tighten(nwc::fe_from_words(w));
}

// out: per element 4 x 8 words (mul, sq, add, sub) of fe32, canonical; mism: mismatches vs fe10
__global__ void k_check(const u32* x, const u32* y, u64 n, u32* out, unsigned long long* mism) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fe32 a = ld32(x + 8 * i), b = ld32(y + 8 * i);
  const fe32 r[4] = {fe32x::fe32_canon(fe32x::fe32_mul(a, b)), fe32x::fe32_canon(fe32x::fe32_sq(a)),
                     fe32x::fe32_canon(fe32x::fe32_add(a, b)), fe32x::fe32_canon(fe32x::fe32_sub(a, b))};
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 8; ++j) out[(4 * i + k) * 8 + j] = r[k].v[j];
  // the 10-limb field sees the low 255 bits; compare where both hold the same value
  if ((x[8 * i + 7] >> 31) == 0 && (y[8 * i + 7] >> 31) == 0) {
    const fe a10 = ld10(x + 8 * i), b10 = ld10(y + 8 * i);
    const fe s[4] = {nwc::fe_mul(a10, b10), nwc::fe_sq(a10), nwc::fe_add(a10, b10), nwc::fe_sub(a10, b10)};
    unsigned bad = 0;
    for (int k = 0; k < 4; ++k) {
      u32 w[8];
      nwc::fe_to_words(s[k], w);
      for (int j = 0; j < 8; ++j) bad |= w[j] != r[k].v[j];
    }
    if (bad) atomicAdd(mism, 1ull);
  }
}

template <int OP>   // 0 fe_mul, 1 fe_sq, 2 fe32_mul, 3 fe32_sq, 4 fe_add+fe_sub pair, 5 fe32 add+sub pair
__global__ __launch_bounds__(256) void k_bench(int iters, const u32* seed, u32* sink) {
  const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  u32 w[8];
  for (int j = 0; j < 8; ++j) w[j] = seed[j] ^ (u32)(t * 2654435761u + j);
  w[7] &= 0x7FFFFFFFu;
  if constexpr (OP == 0 || OP == 1 || OP == 4) {
    fe y = nwc::fe_tighten(nwc::fe_from_words(w));
    w[0] ^= 0x5A5A5A5Au;
    fe x0 = nwc::fe_tighten(nwc::fe_from_words(w));
    w[1] ^= 0x3C3C3C3Cu;
    fe x1 = nwc::fe_tighten(nwc::fe_from_words(w));
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
      if constexpr (OP == 0) { x0 = nwc::fe_mul(x0, y); x1 = nwc::fe_mul(x1, y); }
      else if constexpr (OP == 1) { x0 = nwc::fe_sq(x0); x1 = nwc::fe_sq(x1); }
      else { x0 = nwc::fe_sub(nwc::fe_add(x0, y), x1); x1 = nwc::fe_sub(nwc::fe_add(x1, y), x0); }
    }
    for (int j = 0; j < 10; ++j) sink[t * 20 + j] = (u32)x0.v[j] ^ (u32)x1.v[j];
  } else {
    fe32 y;
    for (int j = 0; j < 8; ++j) y.v[j] = w[j];
    w[0] ^= 0x5A5A5A5Au;
    fe32 x0, x1;
    for (int j = 0; j < 8; ++j) x0.v[j] = w[j];
    w[1] ^= 0x3C3C3C3Cu;
    for (int j = 0; j < 8; ++j) x1.v[j] = w[j];
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
      if constexpr (OP == 2) { x0 = fe32x::fe32_mul(x0, y); x1 = fe32x::fe32_mul(x1, y); }
      else if constexpr (OP == 3) { x0 = fe32x::fe32_sq(x0); x1 = fe32x::fe32_sq(x1); }
      else { x0 = fe32x::fe32_sub(fe32x::fe32_add(x0, y), x1); x1 = fe32x::fe32_sub(fe32x::fe32_add(x1, y), x0); }
    }
    for (int j = 0; j < 8; ++j) sink[t * 20 + j] = x0.v[j] ^ x1.v[j];
  }
}

static u64 rng_state = 0x9E3779B97F4A7C15ull;
static u32 rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (u32)(rng_state >> 16);
}
static const u32 P[8] = {0xFFFFFFEDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};

static void gen(u32* v, int cls) {
  for (int j = 0; j < 8; ++j) v[j] = rnd();
  switch (cls) {
    case 0: v[7] &= 0x7FFFFFFFu; break;                                   // < 2^255
    case 1: for (int j = 1; j < 8; ++j) v[j] = P[j];                      // [p, 2^255) or just below p
            v[0] = 0xFFFFFFEDu + (rnd() % 19); break;
    case 2: break;                                                        // any 256-bit value
    case 3: for (int j = 0; j < 8; ++j) v[j] = (rnd() & 1) ? 0xFFFFFFFFu : 0; v[7] &= 0x7FFFFFFFu; break;
    case 4: for (int j = 0; j < 8; ++j) v[j] = 0; v[0] = rnd() % 64; break;   // tiny
    case 5: for (int j = 0; j < 8; ++j) v[j] = 0xFFFFFFFFu; v[0] -= rnd() % 64; break;   // near 2^256
  }
}

int main(int argc, char** argv) {
  const u64 n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1u << 20);
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  std::vector<u32> x(8 * n), y(8 * n);
  for (u64 i = 0; i < n; ++i) {
    const int cx = (i % 16 < 11) ? 0 : (int)(i % 16) - 10, cy = (i % 7 < 5) ? 0 : (int)(i % 7) - 4;
    gen(&x[8 * i], cx % 6);
    gen(&y[8 * i], cy % 6);
  }
  u32 *dx, *dy, *dout;
  unsigned long long* dm;
  CHECK(hipMalloc(&dx, 32 * n));
  CHECK(hipMalloc(&dy, 32 * n));
  CHECK(hipMalloc(&dout, 128 * n));
  CHECK(hipMalloc(&dm, 8));
  CHECK(hipMemcpy(dx, x.data(), 32 * n, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dy, y.data(), 32 * n, hipMemcpyHostToDevice));
  CHECK(hipMemset(dm, 0, 8));
  hipLaunchKernelGGL(k_check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, dy, n, dout, dm);
  CHECK(hipGetLastError());
  unsigned long long mism = 0;
  CHECK(hipMemcpy(&mism, dm, 8, hipMemcpyDeviceToHost));
  u64 compared = 0;
  for (u64 i = 0; i < n; ++i) compared += (x[8 * i + 7] >> 31) == 0 && (y[8 * i + 7] >> 31) == 0;
  // subset for the big-integer check (every class, bit 255 set included)
  const u64 ns = n < 65536 ? n : 65536;
  std::vector<u32> out(32 * ns);
  CHECK(hipMemcpy(out.data(), dout, 128 * ns, hipMemcpyDeviceToHost));
  if (FILE* f = fopen("/tmp/fe32_sub.bin", "wb")) {
    fwrite(&ns, 8, 1, f);
    fwrite(x.data(), 32, ns, f);
    fwrite(y.data(), 32, ns, f);
    fwrite(out.data(), 128, ns, f);
    fclose(f);
  }
  // throughput
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  u32 *dseed, *dsink;
  CHECK(hipMalloc(&dseed, 32));
  CHECK(hipMemcpy(dseed, x.data(), 32, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&dsink, (size_t)4 * cus * 256 * 20 * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[6] = {"fe_mul", "fe_sq", "fe32_mul", "fe32_sq", "fe_add_sub", "fe32_add_sub"};
  printf("{\"n_check\": %llu, \"compared_vs_fe10\": %llu, \"mismatches_vs_fe10\": %llu, \"iters\": %d, \"cus\": %d, \"rates\": {",
         (unsigned long long)n, (unsigned long long)compared, mism, iters, cus);
  for (int op = 0; op < 6; ++op) {
    printf("%s\"%s\": {", op ? ", " : "", names[op]);
    for (int wps = 1; wps <= 4; wps *= 2) {
      const unsigned grid = (unsigned)(wps * cus);   // 256-thread blocks: one wave per SIMD each
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(e0));
        switch (op) {
          case 0: hipLaunchKernelGGL(k_bench<0>, dim3(grid), dim3(256), 0, 0, iters, dseed, dsink); break;
          case 1: hipLaunchKernelGGL(k_bench<1>, dim3(grid), dim3(256), 0, 0, iters, dseed, dsink); break;
          case 2: hipLaunchKernelGGL(k_bench<2>, dim3(grid), dim3(256), 0, 0, iters, dseed, dsink); break;
          case 3: hipLaunchKernelGGL(k_bench<3>, dim3(grid), dim3(256), 0, 0, iters, dseed, dsink); break;
          case 4: hipLaunchKernelGGL(k_bench<4>, dim3(grid), dim3(256), 0, 0, iters, dseed, dsink); break;
          case 5: hipLaunchKernelGGL(k_bench<5>, dim3(grid), dim3(256), 0, 0, iters, dseed, dsink); break;
        }
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep && ms < best) best = ms;
      }
      const double ops = 2.0 * iters * grid * 256;   // two chains per lane
      printf("%s\"%d_waves_per_simd\": {\"ms\": %.3f, \"Gops\": %.2f, \"ns_per_op_per_cu\": %.4f}", wps > 1 ? ", " : "", wps,
             best, ops / (best * 1e-3) / 1e9, best * 1e6 / (ops / cus));
    }
    printf("}");
  }
  printf("}}\n");
  return mism ? 1 : 0;
}
