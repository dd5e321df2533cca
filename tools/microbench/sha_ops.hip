// Issue rate of the SHA-512 building blocks on gfx950 at 1 and 2 waves per SIMD (4 / 8 waves per
// CU): is a 64-bit add cheaper as one v_lshl_add_u64 or as a v_add_co_u32 + v_addc_co_u32 pair?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 16384;
constexpr int CH = 8;

#define K64(NAME, BODY)                                                                   \
__global__ void NAME(uint32_t* out, uint32_t seed) {                                      \
  uint32_t lo[CH], hi[CH]; uint32_t b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;   \
  uint64_t c64 = ((uint64_t)c << 32) | b;                                                 \
  _Pragma("unroll") for (int i = 0; i < CH; ++i) { lo[i] = seed + i * 7919u + threadIdx.x; hi[i] = lo[i] * 5u; } \
  for (int it = 0; it < ITERS; ++it) {                                                    \
    _Pragma("unroll") for (int i = 0; i < CH; ++i) { BODY; }                              \
  }                                                                                       \
  uint32_t r = 0; _Pragma("unroll") for (int i = 0; i < CH; ++i) r ^= lo[i] ^ hi[i];      \
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                         \
}
#define PAIR ((uint64_t)hi[i] << 32 | lo[i])
K64(k_lshl_add_u64, { uint64_t v = PAIR; asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(v) : "v"(c64)); lo[i] = (uint32_t)v; hi[i] = (uint32_t)(v >> 32); })
K64(k_addco_pair, asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(lo[i]), "+v"(hi[i]) : "v"(b), "v"(c) : "vcc"))
K64(k_alignbit2, asm volatile("v_alignbit_b32 %0, %0, %2, 13\n\tv_alignbit_b32 %1, %1, %2, 7" : "+v"(lo[i]), "+v"(hi[i]) : "v"(b)))
K64(k_bitop3_2, asm volatile("v_bitop3_b32 %0, %0, %2, %3 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0x96" : "+v"(lo[i]), "+v"(hi[i]) : "v"(b), "v"(c)))
K64(k_mad_u64_u32, { uint64_t v = PAIR; asm volatile("v_mad_u64_u32 %0, s[0:1], %1, 1, %0" : "+v"(v) : "v"(b) : "s0", "s1"); lo[i] = (uint32_t)v; hi[i] = (uint32_t)(v >> 32); })
K64(k_mad_i64_i32, { uint64_t v = PAIR; asm volatile("v_mad_i64_i32 %0, s[0:1], %1, %2, %0" : "+v"(v) : "v"(b), "v"(c) : "s0", "s1"); lo[i] = (uint32_t)v; hi[i] = (uint32_t)(v >> 32); })
K64(k_add3_2, asm volatile("v_add3_u32 %0, %0, %2, %3\n\tv_add3_u32 %1, %1, %2, %3" : "+v"(lo[i]), "+v"(hi[i]) : "v"(b), "v"(c)))
K64(k_addco_sgpr, asm volatile("v_add_co_u32_e64 %0, s[2:3], %0, %2\n\tv_add_co_u32_e64 %1, s[4:5], %1, %3\n\tv_addc_co_u32_e64 %0, s[2:3], %0, %3, s[2:3]\n\tv_addc_co_u32_e64 %1, s[4:5], %1, %2, s[4:5]" : "+v"(lo[i]), "+v"(hi[i]) : "v"(b), "v"(c) : "s2", "s3", "s4", "s5"))
K64(k_xor2, asm volatile("v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %3" : "+v"(lo[i]), "+v"(hi[i]) : "v"(b), "v"(c)))

typedef void (*kfn)(uint32_t*, uint32_t);
struct K { const char* name; kfn f; int insts; };

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  K ks[] = {{"v_lshl_add_u64 (1 instr)", k_lshl_add_u64, 1}, {"v_add_co+v_addc (2)", k_addco_pair, 2},
            {"v_alignbit x2", k_alignbit2, 2}, {"v_bitop3 x2", k_bitop3_2, 2}, {"v_xor_b32 x2", k_xor2, 2},
            {"v_mad_u64_u32 (1)", k_mad_u64_u32, 1}, {"v_mad_i64_i32 (1)", k_mad_i64_i32, 1}, {"v_add3_u32 x2", k_add3_2, 2},
            {"2 interleaved add_co/addc (4)", k_addco_sgpr, 4}};
  uint32_t* out;
  for (int wpc : {4, 8, 16}) {
    int threads = 64 * wpc, blocks = cus;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(a));
      const int REP = 3;
      for (int r = 0; r < REP; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r);
      CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
      float ms; CHECK(hipEventElapsedTime(&ms, a, b));
      // cycles per wave-instruction on one SIMD at 2.4 GHz (wave64 VOP2 ideal ~2?, VOP3 ~4?)
      double ops_per_simd = (double)REP * (wpc / 4) * ITERS * CH;   // 64-bit ops per SIMD
      double cyc = ms * 1e-3 * 2.4e9 / ops_per_simd;
      printf("waves/SIMD=%d %-26s %6.2f cycles per 64-bit op (%d instr)\n", wpc / 4, k.name, cyc, k.insts);
    }
    CHECK(hipFree(out));
  }
  return 0;
}
