// Host-side copy helpers shared by the digester (digester.h) and the large host calls
// (nwc_api.hip verify_range): a fixed pool of host threads that fill one pinned stage together,
// and a stager that streams pageable host arrays into HBM through a ring of pinned stages.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

// A fixed set of host threads that fill one pinned stage together (each a contiguous byte range):
// one memcpy thread moves ~30 GB/s, and spawning threads per 32-MB stage costs ~10 % of the fill.
struct CopyPool {
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv, cv_done;
  uint64_t gen = 0;
  unsigned used = 0, pending = 0;
  bool quit = false;
  std::function<void(unsigned)> job;
  void start(unsigned n) {   // n - 1 helpers; the caller is part 0
    for (unsigned i = 1; i < n; ++i)
      th.emplace_back([this, i] {
        uint64_t seen = 0;
        for (;;) {
          std::unique_lock<std::mutex> lk(m);
          cv.wait(lk, [&] { return quit || gen != seen; });
          if (quit) return;
          seen = gen;
          if (i >= used) continue;
          auto f = job;
          lk.unlock();
          f(i);
          lk.lock();
          if (--pending == 0) cv_done.notify_one();
        }
      });
  }
  // f(0 .. parts-1), part 0 on the calling thread
  void run(unsigned parts, const std::function<void(unsigned)>& f) {
    parts = std::min<unsigned>(parts, (unsigned)th.size() + 1);
    if (parts <= 1) { f(0); return; }
    {
      std::lock_guard<std::mutex> lk(m);
      job = f;
      used = parts;
      pending = parts - 1;
      ++gen;
    }
    cv.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m);
    cv_done.wait(lk, [&] { return pending == 0; });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(m);
      quit = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
    th.clear();
  }
  // a pool still running at process exit (its owner's context was never shut down) is stopped
  // here: destroying a joinable std::thread would call std::terminate
  ~CopyPool() { stop(); }
};

// Pageable host arrays into device memory at the pinned-DMA rate.  hipMemcpyAsync from pageable
// memory bounces through the runtime's own staging at ~20 GB/s (config 3 through
// nwc_verify_batch_many: 670 MB of keys and signatures in 31 ms); here `threads` host threads fill a
// 32-MB pinned stage (ordinary cached pages) while the DMA engine drains the previous ones, four
// in rotation.  put() queues a copy (split across stages as they fill); flush() sends the stage
// being filled.  Every copy goes out on `stream` in put() order.
struct HostStager {
  static constexpr size_t STAGE = 32u << 20;
  static constexpr int NST = 4;
  struct Seg { uint8_t* dst; const uint8_t* src; size_t len, off; };
  CopyPool pool;
  uint8_t* stage[NST] = {};
  hipEvent_t ev[NST] = {};
  bool used[NST] = {};
  int cur = 0;
  size_t fill = 0;
  // bytes at which put() flushes the current stage: FIRST after reset(), doubling per flush up
  // to STAGE, so the first DMA starts after a short fill instead of a whole stage's
  static constexpr size_t FIRST = 1u << 20;
  size_t limit = FIRST;
  std::vector<Seg> segs;
  hipStream_t stream = nullptr;

  // At process exit without nwc_shutdown the pool's threads are stopped (CopyPool's destructor);
  // the pinned stages are left to the process teardown (the HIP runtime may be gone by then).
  ~HostStager() = default;

  hipError_t init(hipStream_t s, unsigned threads) {
    stream = s;
    pool.start(threads);
    for (int k = 0; k < NST; ++k) {
      if (hipError_t e = hipHostMalloc(&stage[k], STAGE, hipHostMallocNonCoherent)) return e;
      if (hipError_t e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming)) return e;
    }
    return hipSuccess;
  }
  void release() {
    pool.stop();
    for (int k = 0; k < NST; ++k) {
      if (ev[k]) (void)hipEventSynchronize(ev[k]);
      if (stage[k]) (void)hipHostFree(stage[k]);
      if (ev[k]) (void)hipEventDestroy(ev[k]);
      stage[k] = nullptr;
      ev[k] = nullptr;
    }
  }
  // drop copies queued by a call that failed before its flush (their sources are gone)
  void reset() {
    fill = 0;
    limit = FIRST;
    segs.clear();
  }
  hipError_t put(uint8_t* dst, const uint8_t* src, size_t len) {
    while (len) {
      if (fill >= limit)
        if (hipError_t e = flush()) return e;
      const size_t take = std::min(len, limit - fill);
      segs.push_back(Seg{dst, src, take, fill});
      fill += take;
      dst += take;
      src += take;
      len -= take;
    }
    return hipSuccess;
  }
  hipError_t flush() {
    if (fill == 0) return hipSuccess;
    if (used[cur])
      if (hipError_t e = hipEventSynchronize(ev[cur])) return e;   // its previous DMA has landed
    uint8_t* const st = stage[cur];
    const size_t total = fill;
    const unsigned parts = (unsigned)std::max<size_t>(1, std::min<size_t>(pool.th.size() + 1, total / (1u << 20)));
    const size_t per = (total + parts - 1) / parts;
    pool.run(parts, [&](unsigned t) {   // thread t copies stage bytes [lo, hi)
      const size_t lo = (size_t)t * per, hi = std::min(total, lo + per);
      for (const Seg& g : segs) {
        const size_t a = std::max(lo, g.off), b = std::min(hi, g.off + g.len);
        if (a < b) std::memcpy(st + a, g.src + (a - g.off), b - a);
      }
    });
    for (const Seg& g : segs)
      if (hipError_t e = hipMemcpyAsync(g.dst, st + g.off, g.len, hipMemcpyHostToDevice, stream)) return e;
    if (hipError_t e = hipEventRecord(ev[cur], stream)) return e;
    used[cur] = true;
    cur = (cur + 1) % NST;
    fill = 0;
    limit = std::min(STAGE, 2 * limit);
    segs.clear();
    return hipSuccess;
  }
};

}  // namespace
