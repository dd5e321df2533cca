// Integer-VALU throughput microbenchmark for gfx950 (MI355X).
// Measures issue throughput of the instructions the GF(2^255-19) and SHA-512
// kernels are built from, to freeze the int-VALU roofline.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 8192;
constexpr int CH = 8;   // independent chains per lane

// Each kernel: CH independent chains, ITERS iterations, 1 instruction per chain per iter.
#define KERNEL32(NAME, ASM)                                                        \
__global__ void NAME(uint32_t* out, uint32_t seed) {                               \
  uint32_t v[CH]; uint32_t b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;     \
  _Pragma("unroll") for (int i = 0; i < CH; ++i) v[i] = seed + i * 7919u + threadIdx.x; \
  for (int it = 0; it < ITERS; ++it) {                                             \
    _Pragma("unroll") for (int i = 0; i < CH; ++i) { asm volatile(ASM : "+v"(v[i]) : "v"(b), "v"(c)); } \
  }                                                                                \
  uint32_t r = 0; _Pragma("unroll") for (int i = 0; i < CH; ++i) r ^= v[i];        \
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                  \
}

KERNEL32(k_add_u32,     "v_add_u32 %0, %0, %1")
KERNEL32(k_add3_u32,    "v_add3_u32 %0, %0, %1, %2")
KERNEL32(k_xor_b32,     "v_xor_b32 %0, %0, %1")
KERNEL32(k_alignbit,    "v_alignbit_b32 %0, %0, %1, 13")
KERNEL32(k_bfi,         "v_bfi_b32 %0, %0, %1, %2")
KERNEL32(k_mul_lo_u32,  "v_mul_lo_u32 %0, %0, %1")
KERNEL32(k_mul_hi_u32,  "v_mul_hi_u32 %0, %0, %1")
KERNEL32(k_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL32(k_mul_hi_u24,  "v_mul_hi_u32_u24 %0, %0, %1")
KERNEL32(k_perm,        "v_perm_b32 %0, %0, %1, %2")
KERNEL32(k_dot2_u16,    "v_dot2_u32_u16 %0, %0, %1, %2")
KERNEL32(k_addco,       "v_add_co_u32 %0, vcc, %0, %1")

#define KERNEL64(NAME, ASM)                                                        \
__global__ void NAME(uint32_t* out, uint32_t seed) {                               \
  uint64_t v[CH]; uint32_t b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;     \
  uint64_t c64 = ((uint64_t)c << 32) | b;                                          \
  _Pragma("unroll") for (int i = 0; i < CH; ++i) v[i] = seed + i * 7919ull + threadIdx.x; \
  for (int it = 0; it < ITERS; ++it) {                                             \
    _Pragma("unroll") for (int i = 0; i < CH; ++i) { asm volatile(ASM : "+v"(v[i]) : "v"(b), "v"(c64)); } \
  }                                                                                \
  uint64_t r = 0; _Pragma("unroll") for (int i = 0; i < CH; ++i) r ^= v[i];        \
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r ^ (uint32_t)(r >> 32);  \
}

KERNEL64(k_lshl_add_u64,"v_lshl_add_u64 %0, %0, 1, %2")
KERNEL64(k_fma_f64,     "v_fma_f64 %0, %0, %2, %0")
KERNEL64(k_lshlrev_b64, "v_lshlrev_b64 %0, 3, %0")
KERNEL64(k_add_f64,     "v_add_f64 %0, %0, %2")

__global__ void k_mad_u64_u32(uint32_t* out, uint32_t seed) {
  uint64_t v[CH]; uint32_t b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
  _Pragma("unroll") for (int i = 0; i < CH; ++i) v[i] = seed + i * 7919ull + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
    _Pragma("unroll") for (int i = 0; i < CH; ++i) { asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(v[i]) : "v"(b), "v"(c) : "s0", "s1"); }
  }
  uint64_t r = 0; _Pragma("unroll") for (int i = 0; i < CH; ++i) r ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r ^ (uint32_t)(r >> 32);
}

__global__ void k_fma_f32(uint32_t* out, uint32_t seed) {
  float v[CH]; float b = (float)(seed ^ threadIdx.x) * 1e-9f, c = 1.0f;
  _Pragma("unroll") for (int i = 0; i < CH; ++i) v[i] = (float)i;
  for (int it = 0; it < ITERS; ++it) {
    _Pragma("unroll") for (int i = 0; i < CH; ++i) { asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(b), "v"(c)); }
  }
  float r = 0; _Pragma("unroll") for (int i = 0; i < CH; ++i) r += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(r);
}

typedef void (*kfn)(uint32_t*, uint32_t);
struct K { const char* name; kfn f; };

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  K ks[] = {
    {"v_add_u32", k_add_u32}, {"v_add3_u32", k_add3_u32}, {"v_xor_b32", k_xor_b32},
    {"v_alignbit_b32", k_alignbit}, {"v_bfi_b32", k_bfi}, {"v_mul_lo_u32", k_mul_lo_u32},
    {"v_mul_hi_u32", k_mul_hi_u32}, {"v_mad_u32_u24", k_mad_u32_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u24},
    {"v_perm_b32", k_perm}, {"v_dot2_u32_u16", k_dot2_u16}, {"v_add_co_u32", k_addco},
    {"v_mad_u64_u32", k_mad_u64_u32}, {"v_lshl_add_u64", k_lshl_add_u64}, {"v_fma_f64", k_fma_f64},
    {"v_lshlrev_b64", k_lshlrev_b64}, {"v_add_f64", k_add_f64}, {"v_fma_f32", k_fma_f32},
  };
  int cus = p.multiProcessorCount;
  uint32_t* out; 
  for (int wpc : {8, 16, 32}) {
    int threads = 256, blocks = cus * wpc / 4;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(a));
      const int REP = 5;
      for (int r = 0; r < REP; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r);
      CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
      float ms; CHECK(hipEventElapsedTime(&ms, a, b));
      double insts = (double)REP * blocks * threads * ITERS * CH;   // lane-instructions
      double rate = insts / (ms * 1e-3);                             // lane-ops / s
      double per_clk_cu = rate / (cus * 2.4e9);                      // lanes per clock per CU at 2.4 GHz
      printf("waves/CU=%2d %-18s %8.2f Tlane-op/s  %6.1f lane-op/clk/CU (128 = full rate)\n", wpc, k.name, rate * 1e-12, per_clk_cu);
    }
    CHECK(hipFree(out));
  }
  return 0;
}
