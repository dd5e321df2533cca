// The worker's batch digests behind a Processor-shaped queue (worker/src/processor.rs:35-55).
//
// The reference's Processor task takes one batch off its channel, hashes it
// (`Sha512::digest(&batch)[..32]`, :38), stores it and sends the digest on.  A GPU digest only pays
// for many batches at once (one batch is a 3,970-block chain on one lane, ~30 ms), so
// the device-side Processor drains its channel instead: a drain thread takes the first batch, then
// whatever else arrives within `max_wait_us` (up to `max_group` batches), and digests the group with
// one launch.  Results come back in submission order.  A group that fails on the device comes
// back too: its tags with the error code (never as digests), and the digester then refuses new
// batches (the error is sticky, as a HIP context error is).
//
// Device memory: the group's bytes live in one device buffer, at most NWC_DIGEST_MAX_BYTES
// (16 GiB) per launch -- a larger group is cut into launches of at most that size -- and a buffer
// larger than NWC_DIGEST_KEEP_BYTES (1 GiB) is released after its group, so one 100k-batch group
// does not keep 50 GB resident (nwc_memory_info reports what a digester holds).
//
// Receive arena (nwc_digester_arena): batches the caller placed in the digester's pinned arena are
// DMA'd into the arena's device mirror while their group is still being collected (runs of >= 8 MB),
// and the kernel reads them there; the stage path below is skipped for such a group.
//
// Data path per group: the borrowed batches are gathered into NWC_DIGEST_STAGES (4) pinned 32-MB
// stages in rotation (16-byte-aligned starts, the kernel's dwordx4 path; each stage filled by a
// fixed pool of up to 8 host threads) and DMA'd on the digester's own stream into one device
// buffer while the next stages are filled -- a stage as soon as all of its batches have arrived,
// while the group is still being collected; then k_sha512_digest32[_sched] over the group
// and one D2H of 32 bytes per batch.  The digester has its own stream and buffers (it does not
// serialise with verification calls on the device's context).  Included by nwc_api.hip.
#pragma once
#include <array>
#include <atomic>
#include <deque>

namespace {

struct Digester {
  struct Item { const uint8_t* p; size_t len; uint64_t tag; int status = 0; };
  uint32_t max_group, max_wait_us;
  int hip_id;
  size_t max_bytes = (size_t)16 << 30;   // device bytes per launch (NWC_DIGEST_MAX_BYTES)
  size_t keep_bytes = (size_t)1 << 30;   // device buffer kept between groups (NWC_DIGEST_KEEP_BYTES)
  uint64_t fail_group = 0;               // test hook (NWC_DIGEST_FAIL_GROUP): group k (1-based) fails
  unsigned copy_threads = 8;        // host threads filling a pinned stage (NWC_DIGEST_COPY_THREADS)
  bool timing = false;              // NWC_DIGEST_TIMING: per-group fill / DMA-wait times on stderr
  std::mutex mu;
  std::condition_variable cv_in, cv_out, cv_idle;
  unsigned pollers = 0;            // threads inside nwc_digester_poll (destroy waits for them)
  std::deque<Item> in;
  std::deque<Item> out;            // tag + status + digest (p unused)
  std::deque<std::array<uint8_t, 32>> out_dig;
  int err = 0;
  std::string err_msg;
  bool stop = false;
  uint64_t groups = 0, batches = 0, bytes = 0, submitted = 0, launched = 0;
  uint64_t returned = 0;           // results pushed to `out` (ok or failed); submitted - returned are in flight
  std::thread th;
  CopyPool pool;
  std::chrono::steady_clock::time_point t_group;   // first batch of the current group taken (timing)
  // device side (touched by the drain thread only)
  hipStream_t stream = nullptr;
  static constexpr size_t STAGE = 32u << 20;
  static constexpr int MAX_STAGES = 8;
  int nstages = 4;                  // pinned stages in rotation (NWC_DIGEST_STAGES, 2..8)
  uint8_t* stage[MAX_STAGES] = {};
  hipEvent_t stage_ev[MAX_STAGES] = {};
  uint8_t* ddata = nullptr;
  std::atomic<size_t> ddata_cap{0};
  uint64_t* dse = nullptr;        // starts then ends
  uint8_t* dout = nullptr;
  std::atomic<size_t> k_cap{0};
  uint64_t* hse = nullptr;        // pinned starts/ends
  uint8_t* hout = nullptr;        // pinned digests
  // receive arena (nwc_digester_arena): pinned host memory the caller writes batches into; a group
  // whose batches all lie in it, packed at 16-byte-rounded strides, is DMA'd without a stage fill
  uint8_t* arena = nullptr;
  size_t arena_size = 0;
  // its device mirror: arena bytes [o, o + len) of a submitted batch are DMA'd to darena + o while
  // the drain thread is still collecting the group, so a group of arena batches launches as soon
  // as it closes (drain thread only; allocated at the first such group, arena_size bytes)
  uint8_t* darena = nullptr;
  std::atomic<size_t> darena_cap{0};
  std::atomic<uint64_t> direct_groups{0};

  int init() {
    pool.start(copy_threads);
    HIP_TRY(hipSetDevice(hip_id));
    HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (int s = 0; s < nstages; ++s) {
      // non-coherent: ordinary cached host pages for the copy threads (the default, fine-grained
      // kind is uncached for CPU stores and caps the gather at a few GB/s); the DMA reads it
      HIP_TRY(hipHostMalloc(&stage[s], STAGE, hipHostMallocNonCoherent));
      HIP_TRY(hipEventCreateWithFlags(&stage_ev[s], hipEventDisableTiming));
    }
    return 0;
  }
  void release() {
    pool.stop();
    (void)hipSetDevice(hip_id);
    if (stream) (void)hipStreamSynchronize(stream);
    for (int s = 0; s < MAX_STAGES; ++s) {
      if (stage[s]) (void)hipHostFree(stage[s]);
      if (stage_ev[s]) (void)hipEventDestroy(stage_ev[s]);
    }
    if (ddata) (void)hipFree(ddata);
    if (dse) (void)hipFree(dse);
    if (dout) (void)hipFree(dout);
    if (hse) (void)hipHostFree(hse);
    if (hout) (void)hipHostFree(hout);
    if (arena) (void)hipHostFree(arena);
    if (darena) (void)hipFree(darena);
    if (stream) (void)hipStreamDestroy(stream);
  }

  // device bytes the batch takes in a group's buffer (16-byte aligned starts)
  static uint64_t padded(size_t len) { return (len + 15) & ~(uint64_t)15; }

  // the group being collected: all of its batches in the arena so far, and how many of them have
  // had their DMA queued (drain thread only)
  bool mirrored = false;
  size_t mirrored_sent = 0;
  uint64_t mirror_pending = 0;   // bytes of g[mirrored_sent..]
  // collected arena bytes are DMA'd in runs of at least this much (many small DMAs of single
  // 500-KB batches ran at half the copy engine's rate); the rest when the group closes
  static constexpr uint64_t MIRROR_CHUNK = 8u << 20;
  uint64_t mirror_runs = 0;    // DMAs queued for the current group (NWC_DIGEST_TIMING)
  int pending_err = 0;
  bool in_arena(const Item& it) const {
    return it.len == 0 || (arena && it.p >= arena && (size_t)(it.p - arena) <= arena_size &&
                           it.len <= arena_size - (size_t)(it.p - arena));
  }
  // Queues the DMAs of g[sent..] (arena batches) into the arena's device mirror at their arena
  // offsets: one DMA per run of batches adjacent in the arena (gaps under 256 bytes are copied
  // along).  Drain thread only.
  int stream_arena(const std::vector<Item>& g, size_t& sent) {
    if (!darena) {
      HIP_TRY(hipMalloc(&darena, arena_size));
      darena_cap = arena_size;
    }
    size_t i = sent;
    while (i < g.size()) {
      if (g[i].len == 0) { ++i; continue; }
      const size_t o = (size_t)(g[i].p - arena);
      size_t e = o + g[i].len, j = i + 1;
      for (; j < g.size(); ++j) {
        if (g[j].len == 0) continue;
        const size_t oj = (size_t)(g[j].p - arena);
        if (oj < e || oj > e + 256) break;
        e = oj + g[j].len;
      }
      HIP_TRY(hipMemcpyAsync(darena + o, arena + o, e - o, hipMemcpyHostToDevice, stream));
      ++mirror_runs;
      i = j;
    }
    sent = g.size();
    return 0;
  }

  // Stage gathering of a group that is not in the arena, also started while the group is still
  // being collected: the device layout's offsets of the batches collected so far (16-byte aligned,
  // in arrival order), the bytes [0, gpos) already gathered into stages and queued for DMA, and the
  // stage rotation.  Drain thread only; reset at each group's first batch.
  std::vector<uint64_t> gstart;
  uint64_t gtotal = 0, gpos = 0;
  size_t gfirst = 0;   // first batch that may overlap [gpos, ...)
  int gstage = 0;
  bool gused[MAX_STAGES] = {};
  double t_wait = 0, t_fill = 0;
  void group_reset() {
    gstart.clear();
    gtotal = gpos = 0;
    gfirst = 0;
    gstage = 0;
    for (bool& u : gused) u = false;   // the previous group's DMAs have landed (stream synchronised)
    t_wait = t_fill = 0;
  }
  void group_note(const Item& it) {
    gstart.push_back(gtotal);
    gtotal += padded(it.len);
  }
  // The group's device buffer holds [0, need) (+16 bytes of slack): a larger one keeps the bytes
  // gathered so far, [0, gpos).  While the group grows (stages gathered during its collection) the
  // buffer at least doubles; for a group's final size it gets a quarter of headroom, never past the
  // per-launch cap.
  int ensure_ddata(uint64_t need, bool growing) {
    if (need + 16 <= ddata_cap) return 0;
    const size_t grown = growing ? std::max<size_t>(2 * ddata_cap.load(), (size_t)64 << 20) : (need + 16) + (need + 16) / 4;
    const size_t cap = std::max<size_t>(need + 16, std::min<size_t>(grown, max_bytes + 16));
    uint8_t* nd = nullptr;
    HIP_TRY(hipMalloc(&nd, cap));
    if (ddata) {
      if (gpos) HIP_TRY(hipMemcpyAsync(nd, ddata, gpos, hipMemcpyDeviceToDevice, stream));
      HIP_TRY(hipStreamSynchronize(stream));   // the old buffer's DMAs and this copy are done
      HIP_TRY(hipFree(ddata));
    }
    ddata = nd;
    ddata_cap = cap;
    return 0;
  }
  // Gathers the device layout's bytes [gpos, end) (at most one stage) of g's batches into the next
  // pinned stage with copy_threads host threads (each a contiguous byte range of the stage) and
  // queues its DMA; the other stages' DMAs stay in flight.
  int gather_stage(const std::vector<Item>& g, uint64_t end) {
    using clk = std::chrono::steady_clock;
    if (int rc = ensure_ddata(end, end < gtotal)) return rc;
    const size_t k = g.size();
    const auto t0 = clk::now();
    if (gused[gstage]) HIP_TRY(hipEventSynchronize(stage_ev[gstage]));   // its previous DMA has landed
    const auto t1 = clk::now();
    t_wait += std::chrono::duration<double>(t1 - t0).count();
    const uint64_t pos = gpos;
    uint8_t* const st = stage[gstage];
    while (gfirst < k && gstart[gfirst] + g[gfirst].len <= pos) ++gfirst;   // batches wholly before pos
    auto copy_range = [&](uint64_t lo, uint64_t hi) {
      // batches overlapping [lo, hi), found from gfirst (starts are ascending)
      size_t i = gfirst;
      while (i < k && gstart[i] + g[i].len <= lo) ++i;
      for (; i < k && gstart[i] < hi; ++i) {
        const uint64_t a0 = std::max<uint64_t>(gstart[i], lo), a1 = std::min<uint64_t>(gstart[i] + g[i].len, hi);
        if (a1 > a0) std::memcpy(st + (a0 - pos), g[i].p + (a0 - gstart[i]), a1 - a0);
      }
    };
    const uint64_t bytes = end - pos;
    const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(copy_threads, (bytes + (2u << 20) - 1) / (2u << 20)));
    const uint64_t per = (bytes + nt - 1) / nt;
    pool.run(nt, [&](unsigned t) {
      const uint64_t lo = pos + t * per;
      if (lo < end) copy_range(lo, std::min<uint64_t>(end, lo + per));
    });
    t_fill += std::chrono::duration<double>(clk::now() - t1).count();
    HIP_TRY(hipMemcpyAsync(ddata + pos, st, bytes, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipEventRecord(stage_ev[gstage], stream));
    gused[gstage] = true;
    gstage = (gstage + 1) % nstages;
    gpos = end;
    return 0;
  }

  // SHA-512[..32] of every batch of the group into out32 (32 bytes each)
  int digest_group(const std::vector<Item>& g, uint8_t* out32) {
    const size_t k = g.size();
    if (fail_group && ++launched == fail_group) return set_err(NWC_ERR_DEVICE, "injected digester failure (NWC_DIGEST_FAIL_GROUP)");
    if (k > k_cap) {
      const size_t nk = std::max(k, 2 * k_cap);
      if (dse) HIP_TRY(hipFree(dse));
      if (dout) HIP_TRY(hipFree(dout));
      if (hse) HIP_TRY(hipHostFree(hse));
      if (hout) HIP_TRY(hipHostFree(hout));
      dse = nullptr; dout = nullptr; hse = nullptr; hout = nullptr; k_cap = 0;
      HIP_TRY(hipMalloc(&dse, 16 * nk));
      HIP_TRY(hipMalloc(&dout, 32 * nk));
      HIP_TRY(hipHostMalloc(&hse, 16 * nk, hipHostMallocDefault));
      HIP_TRY(hipHostMalloc(&hout, 32 * nk, hipHostMallocDefault));
      k_cap = nk;
    }
    if (int rc = pending_err) {   // a DMA of the arena mirror failed while the group was collected
      pending_err = 0;
      return rc;
    }
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    // mirror path: every batch in the receive arena, most of its bytes already on their way into
    // the arena's device mirror (stream_arena, queued while the group was collected): the kernel
    // reads them in place there.  Otherwise the batches are gathered into the group's buffer, the
    // stages not yet gathered while the group was collected now (gather_stage).
    const bool direct = mirrored;
    uint64_t total = 0;
    if (direct) {
      if (int rc = stream_arena(g, mirrored_sent)) return rc;
      for (size_t i = 0; i < k; ++i) {
        hse[i] = g[i].len ? (uint64_t)(g[i].p - arena) : 0;
        hse[k + i] = hse[i] + g[i].len;
      }
      ++direct_groups;
    } else {
      for (size_t i = 0; i < k; ++i) {
        hse[i] = gstart[i];
        hse[k + i] = gstart[i] + g[i].len;
      }
      total = gtotal;
      if (int rc = ensure_ddata(total, false)) return rc;
      while (gpos < total)
        if (int rc = gather_stage(g, std::min<uint64_t>(gpos + STAGE, total))) return rc;
    }
    HIP_TRY(hipMemcpyAsync(dse, hse, 16 * k, hipMemcpyHostToDevice, stream));
    if (int rc = launch_digest(direct ? darena : ddata, dse, dse + k, k, dout, stream)) return rc;
    HIP_TRY(hipMemcpyAsync(hout, dout, 32 * k, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    std::memcpy(out32, hout, 32 * k);
    if (ddata_cap > keep_bytes) {   // a large group's buffer is not kept resident
      HIP_TRY(hipFree(ddata));
      ddata = nullptr;
      ddata_cap = 0;
    }
    if (timing && direct)
      std::fprintf(stderr, "nwc digester: group %zu (arena mirror, %llu DMA runs): gathered in %.2f ms, total %.2f ms\n", k,
                   (unsigned long long)mirror_runs, std::chrono::duration<double>(t_start - t_group).count() * 1e3,
                   std::chrono::duration<double>(clk::now() - t_start).count() * 1e3);
    else if (timing)
      std::fprintf(stderr, "nwc digester: group %zu, %.1f MB: gathered in %.2f ms, fill %.2f ms (%.1f GB/s), waits on DMA %.2f ms, total %.2f ms\n",
                   k, total / 1e6, std::chrono::duration<double>(t_start - t_group).count() * 1e3, t_fill * 1e3,
                   total / std::max(t_fill, 1e-9) / 1e9, t_wait * 1e3,
                   std::chrono::duration<double>(clk::now() - t_start).count() * 1e3);
    return 0;
  }

  void run() {
    (void)hipSetDevice(hip_id);
    std::vector<Item> g;
    std::vector<uint8_t> dig;
    for (;;) {
      g.clear();
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_in.wait(lk, [&] { return stop || !in.empty(); });
        if (in.empty()) return;   // stop, drained
        g.push_back(in.front());
        in.pop_front();
        mirrored = arena != nullptr && in_arena(g.back());
        mirrored_sent = 0;
        mirror_pending = g.back().len;
        mirror_runs = 0;
        group_reset();
        group_note(g.back());
        uint64_t gbytes = padded(g.back().len);
        t_group = std::chrono::steady_clock::now();
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(max_wait_us);
        while (g.size() < max_group) {
          if (in.empty()) {
            if (stop || max_wait_us == 0) break;
            if (!cv_in.wait_until(lk, deadline, [&] { return stop || !in.empty(); })) break;
            if (in.empty()) break;
          }
          // one launch's device bytes stay under max_bytes (a single larger batch goes alone)
          if (gbytes + padded(in.front().len) > max_bytes) break;
          gbytes += padded(in.front().len);
          g.push_back(in.front());
          in.pop_front();
          group_note(g.back());
          if (mirrored && !in_arena(g.back())) mirrored = false;   // a batch outside: gather the group
          if (!mirrored && gtotal - gpos >= STAGE && !pending_err) {
            // gather the stages whose batches have all arrived; the group stays open
            lk.unlock();
            while (!pending_err && gtotal - gpos >= STAGE) pending_err = gather_stage(g, gpos + STAGE);
            lk.lock();
          }
          if (mirrored && (mirror_pending += g.back().len) >= MIRROR_CHUNK && !pending_err) {
            // queue the DMAs of the arena batches collected so far; the group stays open
            lk.unlock();
            pending_err = stream_arena(g, mirrored_sent);
            lk.lock();
            mirror_pending = 0;
          }
        }
      }
      dig.resize(32 * g.size());
      const int rc = digest_group(g, dig.data());
      std::lock_guard<std::mutex> lk(mu);
      if (rc && !err) { err = rc; err_msg = t_err; }
      if (!rc) ++groups;
      // every tag comes back, in order: a failed group's with its error code and no digest
      for (size_t i = 0; i < g.size(); ++i) {
        out.push_back(Item{nullptr, g[i].len, g[i].tag, rc});
        ++returned;
        std::array<uint8_t, 32> a{};
        if (!rc) std::memcpy(a.data(), dig.data() + 32 * i, 32);
        out_dig.push_back(a);
        if (!rc) {
          ++batches;
          bytes += g[i].len;
        }
      }
      cv_out.notify_all();
    }
  }
};

// live digesters (nwc_memory_info reports their device buffers per device)
std::mutex g_dg_mu;
std::vector<Digester*> g_digesters;
void digester_register(Digester* q, bool add) {
  std::lock_guard<std::mutex> lk(g_dg_mu);
  if (add) g_digesters.push_back(q);
  else g_digesters.erase(std::remove(g_digesters.begin(), g_digesters.end(), q), g_digesters.end());
}
uint64_t digester_device_bytes(int hip_id) {
  std::lock_guard<std::mutex> lk(g_dg_mu);
  uint64_t b = 0;
  for (const Digester* q : g_digesters)
    if (q->hip_id == hip_id) b += q->ddata_cap.load() + q->darena_cap.load() + 48 * (uint64_t)q->k_cap.load();
  return b;
}

}  // namespace

extern "C" {

nwc_digester* nwc_digester_create(uint32_t max_group, uint32_t max_wait_us) {
  if (require_init()) return nullptr;
  if (max_group == 0) { set_err(NWC_ERR_ARG, "max_group must be >= 1"); return nullptr; }
  auto* q = new Digester();
  q->max_group = max_group;
  q->max_wait_us = max_wait_us;
  q->hip_id = ctx(t_dev < (int)g_devs.size() ? t_dev : 0)->hip_id;
  if (const char* e = std::getenv("NWC_DIGEST_COPY_THREADS")) q->copy_threads = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("NWC_DIGEST_STAGES")) q->nstages = std::min(Digester::MAX_STAGES, std::max(2, std::atoi(e)));
  q->timing = std::getenv("NWC_DIGEST_TIMING") != nullptr;
  if (const char* e = std::getenv("NWC_DIGEST_MAX_BYTES")) q->max_bytes = std::max<size_t>(1 << 20, std::strtoull(e, nullptr, 10));
  if (const char* e = std::getenv("NWC_DIGEST_KEEP_BYTES")) q->keep_bytes = std::strtoull(e, nullptr, 10);
  if (const char* e = std::getenv("NWC_DIGEST_FAIL_GROUP")) q->fail_group = std::strtoull(e, nullptr, 10);
  if (q->init()) {
    q->release();
    delete q;
    return nullptr;
  }
  q->th = std::thread([q] { q->run(); });
  digester_register(q, true);
  return reinterpret_cast<nwc_digester*>(q);
}

int nwc_digester_submit(nwc_digester* h, const uint8_t* batch, size_t len, uint64_t tag) {
  auto* q = reinterpret_cast<Digester*>(h);
  if (!q) return set_err(NWC_ERR_ARG, "null digester");
  if (len && !batch) return set_err(NWC_ERR_ARG, "null batch");
  {
    std::lock_guard<std::mutex> lk(q->mu);
    if (q->stop) return set_err(NWC_ERR_ARG, "digester is shutting down");
    if (q->err) return set_err(q->err, "digester failed earlier: %s", q->err_msg.c_str());
    q->in.push_back(Digester::Item{batch, len, tag});
    ++q->submitted;
  }
  q->cv_in.notify_one();
  return 0;
}

uint8_t* nwc_digester_arena(nwc_digester* h, size_t bytes) {
  auto* q = reinterpret_cast<Digester*>(h);
  if (!q) { set_err(NWC_ERR_ARG, "null digester"); return nullptr; }
  std::lock_guard<std::mutex> lk(q->mu);
  if (q->arena) {
    if (bytes > q->arena_size) { set_err(NWC_ERR_ARG, "the digester's arena exists with %zu bytes", q->arena_size); return nullptr; }
    return q->arena;
  }
  if (bytes == 0) { set_err(NWC_ERR_ARG, "arena size must be > 0"); return nullptr; }
  if (q->submitted) { set_err(NWC_ERR_ARG, "create the arena before the first submit"); return nullptr; }
  // ordinary cached pages for the caller's writes (as the stages); the DMA engine reads them
  const hipError_t e = hipHostMalloc(&q->arena, bytes, hipHostMallocNonCoherent);
  if (e != hipSuccess) {
    q->arena = nullptr;
    set_err(NWC_ERR_DEVICE, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    return nullptr;
  }
  q->arena_size = bytes;
  return q->arena;
}

int nwc_digester_poll(nwc_digester* h, size_t max, uint32_t wait_us, uint64_t* tags, uint8_t* digests32, size_t* n_done) {
  auto* q = reinterpret_cast<Digester*>(h);
  if (!q || !n_done || (max && (!tags || !digests32))) return set_err(NWC_ERR_ARG, "null argument");
  std::unique_lock<std::mutex> lk(q->mu);
  ++q->pollers;
  // the sticky error stands alone only once every submitted batch has come back
  auto drained_err = [&] { return q->err && q->returned == q->submitted; };
  if (wait_us && q->out.empty() && !drained_err() && !q->stop)
    q->cv_out.wait_for(lk, std::chrono::microseconds(wait_us), [&] { return !q->out.empty() || drained_err() || q->stop; });
  // a run of results with one status: digests (rc 0) or a failed group's tags (rc < 0)
  const int status = q->out.empty() ? 0 : q->out.front().status;
  size_t n = 0;
  while (n < max && !q->out.empty() && q->out.front().status == status) {
    tags[n] = q->out.front().tag;
    std::memcpy(digests32 + 32 * n, q->out_dig.front().data(), 32);
    q->out.pop_front();
    q->out_dig.pop_front();
    ++n;
  }
  *n_done = n;
  int rc = 0;
  if (status) rc = set_err(status, "digest group failed: %s", q->err_msg.c_str());
  else if (n == 0 && drained_err()) rc = set_err(q->err, "%s", q->err_msg.c_str());   // sticky, nothing left to hand back
  if (--q->pollers == 0) q->cv_idle.notify_all();
  return rc;
}

int nwc_digester_stats(nwc_digester* h, uint64_t* groups, uint64_t* batches, uint64_t* bytes) {
  auto* q = reinterpret_cast<Digester*>(h);
  if (!q) return set_err(NWC_ERR_ARG, "null digester");
  std::lock_guard<std::mutex> lk(q->mu);
  if (groups) *groups = q->groups;
  if (batches) *batches = q->batches;
  if (bytes) *bytes = q->bytes;
  return 0;
}

int nwc_digester_direct_groups(nwc_digester* h, uint64_t* direct_groups) {
  auto* q = reinterpret_cast<Digester*>(h);
  if (!q || !direct_groups) return set_err(NWC_ERR_ARG, "null argument");
  *direct_groups = q->direct_groups.load();
  return 0;
}

int nwc_digester_destroy(nwc_digester* h) {
  auto* q = reinterpret_cast<Digester*>(h);
  if (!q) return 0;
  {
    std::lock_guard<std::mutex> lk(q->mu);
    q->stop = true;
  }
  q->cv_in.notify_all();
  q->cv_out.notify_all();   // a poller blocked on an empty queue returns now
  if (q->th.joinable()) q->th.join();
  {
    // no thread may still be inside poll when the digester is freed
    std::unique_lock<std::mutex> lk(q->mu);
    q->cv_idle.wait(lk, [&] { return q->pollers == 0; });
  }
  digester_register(q, false);
  const int rc = q->err;
  q->release();
  delete q;
  return rc;
}

}  // extern "C"
