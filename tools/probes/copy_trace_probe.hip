// Which hipMemcpyAsync shapes leave rocprofv3's memory-copy tracer waiting for completions that
// HSA never delivers (verdict r04 item 5)?  No libnwc: plain HIP copies only.
//   probe MODE   MODE: pageable_d2h | pageable_h2d | pinned_d2h | pinned_h2d | big_pinned_h2d |
//                      coherent_d2h | coherent_h2d (hipHostMallocCoherent: libnwc's small-call stage)
// Each mode does 4 copies of its shape, synchronises the stream after each, checks the bytes and
// exits normally.  Run under `rocprofv3 --memory-copy-trace` and read the tool's warnings.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "pageable_d2h";
  const bool big = std::strcmp(mode, "big_pinned_h2d") == 0;
  const size_t n = big ? (size_t)32 << 20 : (size_t)80 << 10;
  const bool coherent = std::strstr(mode, "coherent") != nullptr;
  const bool pinned = coherent || std::strstr(mode, "pinned") != nullptr;
  const bool d2h = std::strstr(mode, "d2h") != nullptr;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void* dev = nullptr;
  CHECK(hipMalloc(&dev, n));
  std::vector<unsigned char> pageable(n);
  unsigned char* host = pageable.data();
  if (pinned)
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&host), n, coherent ? hipHostMallocCoherent : hipHostMallocDefault));
  for (int rep = 0; rep < 4; ++rep) {
    const unsigned char v = (unsigned char)(17 + rep);
    if (d2h) {
      CHECK(hipMemsetAsync(dev, v, n, s));
      CHECK(hipMemcpyAsync(host, dev, n, hipMemcpyDeviceToHost, s));
      CHECK(hipStreamSynchronize(s));
      for (size_t i = 0; i < n; i += 4099)
        if (host[i] != v) { std::fprintf(stderr, "mismatch at %zu\n", i); return 3; }
    } else {
      std::memset(host, v, n);
      CHECK(hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, s));
      CHECK(hipStreamSynchronize(s));
    }
  }
  if (pinned) CHECK(hipHostFree(host));
  CHECK(hipFree(dev));
  CHECK(hipStreamDestroy(s));
  std::printf("%s: 4 copies of %zu bytes ok\n", mode, n);
  return 0;
}
