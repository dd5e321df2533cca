// Host side of libnwc.so: the C ABI declared in include/nwc.h.
//
// One context per HIP device: its own stream, the basepoint table, and a growable staging
// arena.  A per-device mutex makes every entry point thread-safe (the reference calls the
// crypto crate from concurrent tokio tasks: primary/src/core.rs:88-114,
// worker/src/worker.rs:182,227).  Host batch entry points shard independent units
// (signatures, certificates, messages) over all initialised devices with one host thread per
// device; nothing here ever falls back to a CPU path -- a device failure is
// an error code (< 0), never a verdict.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <functional>
#include <thread>
#include <unordered_set>
#include <vector>

#include "nwc.h"
#include "copy_pool.h"
#include "kernels.hip"
#include "launch_keys.h"
#include "messages.h"

namespace {

thread_local std::string t_err;
thread_local int t_dev = 0;

int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  t_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return set_err(NWC_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                     __FILE__, __LINE__);                                                       \
  } while (0)

// Exact 32-byte key lookup with the device's hash and probing (committee_lookup): the host copy
// of a device key cache, so that small host calls can tell before launching whether every key
// is cached.
struct KeyIndex {
  std::vector<nwc::u32> keys;   // 8 words per key
  std::vector<int32_t> slots;   // slot -> key index, -1 empty
  uint32_t mask = 0;
  bool find(const uint8_t* pk) const {
    if (slots.empty()) return false;
    nwc::u32 w[8];
    std::memcpy(w, pk, 32);
    const nwc::u32 h = nwc::committee_hash(w[0], w[1]);
    for (int p = 0; p < nwc::COMMITTEE_MAX_PROBE; ++p) {
      const int32_t idx = slots[(h + p) & mask];
      if (idx < 0) return false;
      if (std::memcmp(&keys[8 * (size_t)idx], w, 32) == 0) return true;
    }
    return false;
  }
  bool all_found(const uint8_t* pks, uint64_t n) const {
    for (uint64_t i = 0; i < n; ++i)
      if (!find(pks + 32 * i)) return false;
    return true;
  }
};

// Open-addressing slot table over the first n keys (load factor <= 1/4, probe length bounded by
// COMMITTEE_MAX_PROBE; a duplicate key keeps its first index).
uint32_t build_slots(const std::vector<nwc::u32>& keys, size_t n, std::vector<int32_t>& table) {
  uint32_t slots = 16;
  while (slots < 4 * n) slots <<= 1;
  for (;;) {
    table.assign(slots, -1);
    bool fits = true;
    for (size_t i = 0; i < n && fits; ++i) {
      const nwc::u32 h = nwc::committee_hash(keys[8 * i], keys[8 * i + 1]);
      int p = 0;
      for (; p < nwc::COMMITTEE_MAX_PROBE; ++p) {
        int32_t& slot = table[(h + p) & (slots - 1)];
        if (slot < 0) { slot = (int32_t)i; break; }
        if (std::memcmp(&keys[8 * slot], &keys[8 * i], 32) == 0) break;   // duplicate key
      }
      fits = p < nwc::COMMITTEE_MAX_PROBE;
    }
    if (fits) return slots;
    slots <<= 1;
  }
}

struct DevCtx {
  int hip_id = 0;
  int cus = 0;
  int verify_blocks_per_cu = 1;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;      // small batch-leaf calls: the keys' torsion test beside the verification
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_msg = nullptr;   // sanitize: k_header_digests done on the side stream
  hipEvent_t ev_count = nullptr; // sanitize: the vote count has reached the host
  // large host calls: input chunks are copied on `xfer` while the previous chunk verifies on
  // `stream` (one event per chunk in flight, created on first use)
  hipStream_t xfer = nullptr;
  std::vector<hipEvent_t> ev_chunk;
  std::vector<hipEvent_t> ev_cnt;      // sanitize: chunk k's vote count copied to the host
  nwc::ge_niels* base_table = nullptr;
  nwc::ge_niels_pad* base24 = nullptr;   // radix-2^24 basepoint tables (2.1 GB)
  nwc::ge_p3* base24_points = nullptr;    // B and 2^141 B
  nwc::ge_niels_pad* comb_base = nullptr;   // radix-256 basepoint comb (528 KB): latency kernel
  nwc::ge_niels_pad* comb16 = nullptr;      // basepoint comb (radix 2^NWC_BCOMB_BITS, 67 MB at 2^16): k_verify_comb
  nwc::ge_p3* comb16_bases = nullptr;       // its window bases 2^(bits w) B (built at init)
  nwc::ge_p3* kb_bases = nullptr;           // key comb window bases (scratch of build_key_combs)
  size_t kb_cap = 0;
  int comb_blocks_per_cu = 1;
  uint8_t* straus_scratch = nullptr;   // k_verify_straus per-lane tables (nwc_dev_verify_batch_straus)
  size_t straus_cap = 0;
  uint8_t* msm_scratch = nullptr;      // k_verify_msm per-wave points and digits (nwc_dev_verify_batch_msm)
  size_t msm_cap = 0;
  uint32_t* msm_stats = nullptr;       // groups passed / failed / key overflow (nwc_msm_stats)
  uint8_t* rs_buf = nullptr;           // dalek's equation per certificate (resolve.h): failing-vote list, certificate states
  size_t rs_cap = 0;
  uint32_t* uc_list = nullptr;     // k_verify_comb: equations whose key is not cached
  uint32_t* uc_count = nullptr;
  bool hold_lists = false;         // a call with a deferred list pending: ensure_scratch does not shrink the lists
  bool tables_ready = false;       // ensure_verify_tables has built the basepoint tables, memo and auto cache
  // k_verify per-lane table slots; reused by every launch, so launches that use it are
  // serialised across streams with `scratch_free` (recorded after each such launch).
  uint8_t* scratch = nullptr;
  size_t scratch_cap = 0;
  uint32_t* fb_list = nullptr;     // lanes whose half-size reduction failed (k_verify_fallback)
  uint32_t* fb_count = nullptr;
  uint8_t* pair_buf = nullptr;      // the paired strict host pipeline: per-chunk fallback counts + lists
  size_t pair_cap = 0;
  uint8_t* sign_buf = nullptr;      // large host calls on the comb path: two chunks' SignRecs
  size_t sign_cap = 0;
  const uint8_t* busy_buf = nullptr;   // a buffer a host pipeline's launches use: never released under it
  uint64_t* stamps = nullptr;      // k_verify<.., STAMP>: 4 words per wave of the resident grid (nwc_diag_verify_clock)
  size_t fb_cap = 0;
  hipEvent_t scratch_free = nullptr;
  // batch-leaf torsion post-pass (k_tors_*): key hash set sized for fb_cap equations
  int32_t* ts_slots = nullptr;
  uint32_t* ts_flag = nullptr;
  uint32_t* ts_uniq = nullptr;
  uint32_t* ts_nuniq = nullptr;
  uint32_t ts_slot_count = 0;
  nwc::u32* km_keys = nullptr;   // torsion memo of uncached keys (KeyMemo), kept for the context's life
  nwc::u32* km_flag = nullptr;
  // committee key cache (nwc_set_committee); buffers replaced only after scratch_free
  nwc::u32* cm_keys = nullptr;
  nwc::u32* cm_flags = nullptr;
  nwc::ge_niels* cm_tables = nullptr;
  nwc::ge_niels_pad* cm_comb = nullptr;   // per-key combs (committees of <= COMB_MAX_KEYS keys)
  int32_t* cm_slots = nullptr;
  uint32_t cm_n = 0, cm_slot_mask = 0;
  size_t cm_bytes = 0;                  // device bytes of the committee cache (nwc_memory_info)
  uint8_t* arena = nullptr;
  size_t arena_cap = 0;
  // config::Committee stake / worker tables (nwc_set_committee_config)
  uint64_t* cc_stakes = nullptr;
  uint32_t* cc_worker_off = nullptr;
  uint32_t* cc_worker_ids = nullptr;
  uint64_t cc_quorum = 0;
  uint32_t cc_n = 0;
  uint8_t* msg_arena = nullptr;   // nwc_sanitize_messages buffers
  size_t msg_arena_cap = 0;
  uint8_t* pinned = nullptr;   // host staging for small calls: one H2D and one D2H per call, or
  uint8_t* pinned_dev = nullptr;   // read in place by the latency kernel through this device pointer
  size_t pinned_cap = 0;
  // auto key cache (NWC_AUTO_KEYS): keys of small host calls outside the committee cache, added
  // with their flags, 129-entry tables and combs the second time they are seen, so that repeated
  // first-sight certificates take the latency kernel; append-only, guarded by mu like the rest
  nwc::u32* ak_keys = nullptr;
  nwc::u32* ak_flags = nullptr;
  nwc::ge_niels* ak_tables = nullptr;
  nwc::ge_niels_pad* ak_comb = nullptr;
  int32_t* ak_slots = nullptr;
  uint32_t ak_n = 0, ak_cap = 0, ak_slot_cap = 0;
  uint32_t ak_evict = 0;                  // next FIFO position once the cache is full
  uint64_t ak_builds = 0, ak_hits = 0;    // insert batches built / calls served from the auto cache
  KeyIndex ak_host;                       // host copy of the auto cache's lookup table
  std::unordered_set<std::string> ak_seen;   // keys seen once (32-byte strings), bounded
  // copy sources of the last auto-cache build, alive until the stream has passed it
  std::vector<nwc::u32> ak_pend_keys;
  std::vector<int32_t> ak_pend_slots;
  bool ak_pending = false;
  // launch keys (launch_keys.h): allocated by the first large batch-leaf launch without a committee
  nwc::LaunchKeys lk{};
  bool lk_alloc = false;
  bool lk_censused = false;           // the first launch-key launch has measured its keys' demand
  uint32_t* lk_demand = nullptr;      // host-mapped demand word (lk.host_demand's host side)
  // large host calls: pageable inputs through pinned stages on `xfer` (created on first use)
  std::unique_ptr<HostStager> stager;
  std::mutex mu;

  int ensure_pinned(size_t bytes) {
    if (bytes <= pinned_cap) return 0;
    if (pinned) { (void)hipHostFree(pinned); pinned = nullptr; pinned_cap = 0; }
    // coherent: the latency kernel's verdict bytes reach the host while it polls them
    HIP_TRY(hipHostMalloc(&pinned, bytes, hipHostMallocCoherent));
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, pinned, 0));
    pinned_dev = static_cast<uint8_t*>(dp);
    pinned_cap = bytes;
    return 0;
  }
  int ensure_arena(size_t bytes) {
    if (bytes <= arena_cap) return 0;
    if (arena) { (void)hipFree(arena); arena = nullptr; arena_cap = 0; }
    size_t cap = bytes + bytes / 4 + (1 << 20);
    HIP_TRY(hipMalloc(&arena, cap));
    arena_cap = cap;
    return 0;
  }
};

// slots of the per-device torsion memo of uncached keys (power of two)
#ifndef NWC_MEMO_SLOTS
#define NWC_MEMO_SLOTS (1u << 16)
#endif
// committees up to this size get per-key combs (20 MB each at radix 2^14); larger ones use the cached ladder
#ifndef NWC_COMB_MAX_KEYS
#define NWC_COMB_MAX_KEYS 1024
#endif

// batches up to this size take the latency kernel (k_verify_comb_wide) on the comb path
// Host calls of at least 2 chunks are pipelined: chunk i+1's inputs cross PCIe while chunk i
// verifies.  A chunk is one full round of resident lanes (2 blocks of 256 per CU x 256 CUs).
#ifndef NWC_HOST_CHUNK
#define NWC_HOST_CHUNK (1u << 17)
#endif
#ifndef NWC_HOST_CHUNK_MAX
#define NWC_HOST_CHUNK_MAX (1u << 20)
#endif
#ifndef NWC_MSG_CHUNK
#define NWC_MSG_CHUNK (24u << 20)   // largest pipelined chunk of nwc_sanitize_messages, bytes of wire messages (A/B: profiles/r05/wire_host.md)
#endif
#ifndef NWC_HOST_CHUNK_GROWTH
#define NWC_HOST_CHUNK_GROWTH 3
#endif
#ifndef NWC_PINNED_STAGE_MAX
#define NWC_PINNED_STAGE_MAX (1u << 20)
#endif
// persistent verify grid: this many blocks per resident block slot
#ifndef NWC_VERIFY_GRID_MULT
#define NWC_VERIFY_GRID_MULT 8
#endif
#ifndef NWC_WIDE_MAX
#define NWC_WIDE_MAX 1024
#endif

std::mutex g_mu;
std::vector<std::unique_ptr<DevCtx>> g_devs;

struct HostCommittee {
  std::mutex mu;
  KeyIndex idx;
  bool all_cached(const uint8_t* pks, uint64_t n) {
    std::lock_guard<std::mutex> lk(mu);
    return idx.all_found(pks, n);
  }
};
HostCommittee g_hcm;

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Carve {
  uint8_t* base;
  size_t off = 0;
  explicit Carve(uint8_t* b) : base(b) {}
  template <class T> T* take(size_t bytes) { T* p = reinterpret_cast<T*>(base + off); off += align256(bytes); return p; }
};

uint32_t auto_keys_cap();
int auto_grow(DevCtx& d, uint32_t ncap);
bool comb16_enabled();

// Test and A/B knobs settable at run time (nwc_diag_set), defaults from the environment read once:
// NWC_STRAUS_NQ (votes per Straus sub-batch, 12) and NWC_FORCE_WINDOWS (half-ladder window count
// forced on every wave, 0 = off).  Atomics: a setter racing a launch gives that launch either value.
struct Knobs {
  std::atomic<uint32_t> straus_nq{12};
  std::atomic<uint32_t> force_windows{0};
  std::atomic<uint32_t> launch_keys{1};   // NWC_LAUNCH_KEYS: 0 = large batch-leaf launches never build launch keys
  std::atomic<uint32_t> msm_group{0};     // NWC_MSM_GROUP: votes per Pippenger group of k_verify_msm (0 = sized per launch)
  std::atomic<uint32_t> msm_adapt{1};     // NWC_MSM_ADAPT: 0 = the equation on every group (no skip policy)
  std::atomic<uint64_t> dalek_seed{0};    // tests: fixed seed of the per-certificate equation's z_i (0 = host CSPRNG)
  Knobs() {
    if (const char* e = std::getenv("NWC_LAUNCH_KEYS")) launch_keys = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("NWC_STRAUS_NQ")) straus_nq = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("NWC_FORCE_WINDOWS")) force_windows = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("NWC_MSM_GROUP")) msm_group = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("NWC_MSM_ADAPT")) msm_adapt = std::atoi(e) != 0;
  }
};
Knobs& knobs() {
  static Knobs k;
  return k;
}

int init_device(DevCtx& d) {
  HIP_TRY(hipSetDevice(d.hip_id));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, d.hip_id));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(NWC_ERR_NO_DEVICE, "device %d is %s; libnwc is built for gfx950 only", d.hip_id, prop.gcnArchName);
  HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&d.scratch_free, hipEventDisableTiming));
  HIP_TRY(hipStreamCreateWithFlags(&d.side, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&d.ev_fork, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&d.ev_join, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&d.ev_msg, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&d.ev_count, hipEventDisableTiming));
  d.cus = prop.multiProcessorCount;
  int bpc = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, reinterpret_cast<const void*>(nwc::k_verify<true, false>), 256, 0));
  d.verify_blocks_per_cu = bpc > 0 ? bpc : 1;
  if (std::getenv("NWC_SHOW_OCCUPANCY")) std::fprintf(stderr, "nwc: k_verify resident blocks per CU %d\n", bpc);
  bpc = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, reinterpret_cast<const void*>(nwc::k_verify_comb), 256, 0));
  d.comb_blocks_per_cu = bpc > 0 ? bpc : 1;
  HIP_TRY(hipMalloc(&d.uc_count, sizeof(uint32_t)));
  HIP_TRY(hipMalloc(&d.fb_count, sizeof(uint32_t)));
  HIP_TRY(hipStreamSynchronize(d.stream));
  return 0;
}

// The verification tables, built by the first call that verifies (or signs) on the device, not at
// nwc_init: a worker process that only digests batches holds none of them (worker/src/worker.rs:
// 182-188 -- workers and a primary share the host's GPUs).  Built on d.stream and waited for once,
// so launches on any stream after it see them.  Caller holds d.mu and has set the device.
int ensure_verify_tables(DevCtx& d) {
  if (d.tables_ready) return 0;
  HIP_TRY(hipMalloc(&d.comb_base, nwc::BaseComb::per * sizeof(nwc::ge_niels_pad)));
  hipLaunchKernelGGL(nwc::k_build_comb<nwc::BaseComb>, dim3((unsigned)((nwc::BaseComb::per + 255) / 256)), dim3(256), 0, d.stream,
                     (const nwc::u32*)nullptr, 1u, d.comb_base);
  HIP_TRY(hipGetLastError());
  if (comb16_enabled()) {
    // radix-2^22 basepoint comb (3.2 GB): the committee comb kernel and the cold kernel's s B
    HIP_TRY(hipMalloc(&d.comb16, nwc::COMB16_TOTAL * sizeof(nwc::ge_niels_pad)));
    HIP_TRY(hipMalloc(&d.comb16_bases, nwc::COMB16_WINDOWS * sizeof(nwc::ge_p3)));
    hipLaunchKernelGGL(nwc::k_bcomb_bases, dim3(1), dim3(64), 0, d.stream, d.comb16_bases);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(nwc::k_build_comb16, dim3((unsigned)((nwc::COMB16_TOTAL + 255) / 256)), dim3(256), 0, d.stream,
                       d.comb16, (const nwc::ge_p3*)d.comb16_bases);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMalloc(&d.base_table, 2 * 129 * sizeof(nwc::ge_niels)));
  hipLaunchKernelGGL(nwc::k_build_base_table, dim3(5), dim3(64), 0, d.stream, d.base_table);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMalloc(&d.base24, 2 * (size_t)nwc::B24_ENTRIES * sizeof(nwc::ge_niels_pad)));
  HIP_TRY(hipMalloc(&d.base24_points, 2 * sizeof(nwc::ge_p3)));
  hipLaunchKernelGGL(nwc::k_base_pow2, dim3(1), dim3(64), 0, d.stream, d.base24_points);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(nwc::k_build_base_table24, dim3((unsigned)((2 * (size_t)nwc::B24_ENTRIES + 255) / 256)), dim3(256), 0,
                     d.stream, d.base24, (const nwc::ge_p3*)d.base24_points);
  HIP_TRY(hipGetLastError());
  // torsion memo: 64K keys (2.3 MB), all slots empty
  HIP_TRY(hipMalloc(&d.km_keys, 32 * (size_t)NWC_MEMO_SLOTS));
  HIP_TRY(hipMalloc(&d.km_flag, 4 * (size_t)NWC_MEMO_SLOTS));
  HIP_TRY(hipMemsetAsync(d.km_flag, 0xFF, 4 * (size_t)NWC_MEMO_SLOTS, d.stream));
  // auto key cache: the first AUTO_INIT_KEYS keys' arrays (~330 MB), their slot table and the key
  // comb builder's scratch are allocated here, so the call that first fills the cache only
  // queues its build (growth beyond this is stream-ordered, auto_grow)
  if (const uint32_t acap = auto_keys_cap()) {
    if (int rc = auto_grow(d, std::min<uint32_t>(acap, 16u))) return rc;
    d.ak_slot_cap = 64;
    while (d.ak_slot_cap < 8 * std::min<uint32_t>(acap, 16u)) d.ak_slot_cap <<= 1;
    HIP_TRY(hipMalloc(&d.ak_slots, 4 * (size_t)d.ak_slot_cap));
    if (!d.kb_bases) {
      d.kb_cap = 64 * (size_t)nwc::KeyComb::windows;
      HIP_TRY(hipMalloc(&d.kb_bases, d.kb_cap * sizeof(nwc::ge_p3)));
    }
  }
  HIP_TRY(hipStreamSynchronize(d.stream));
  d.tables_ready = true;
  return 0;
}

DevCtx* ctx(int i) {
  if (i < 0 || i >= (int)g_devs.size()) return nullptr;
  return g_devs[i].get();
}

int require_init() {
  if (g_devs.empty()) return set_err(NWC_ERR_NOT_INIT, "nwc_init has not been called (or found no device)");
  return 0;
}

// Per-key combs of m keys (KeyComb) into out: window bases first, then one lane per entry.  The
// bases are re-allocated stream-ordered when a larger build needs more.
int build_key_combs(DevCtx& d, const nwc::u32* keys, uint32_t m, nwc::ge_niels_pad* out) {
  if (m == 0) return 0;
  const size_t need = (size_t)m * nwc::KeyComb::windows;
  if (need > d.kb_cap) {
    // stream-ordered: the old bases are freed behind the launches that read them
    if (d.kb_bases) HIP_TRY(hipFreeAsync(d.kb_bases, d.stream));
    d.kb_bases = nullptr;
    d.kb_cap = 0;
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&d.kb_bases), need * sizeof(nwc::ge_p3), d.stream));
    d.kb_cap = need;
  }
  hipLaunchKernelGGL(nwc::k_comb_key_bases<nwc::KeyComb>, dim3((m + 63) / 64), dim3(64), 0, d.stream, keys, m, d.kb_bases);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(nwc::k_build_comb_from_bases<nwc::KeyComb>, dim3((unsigned)(d.cus * 8)), dim3(256), 0, d.stream,
                     (const nwc::ge_p3*)d.kb_bases, 0u, m, (const uint32_t*)nullptr, out);
  HIP_TRY(hipGetLastError());
  return 0;
}

// NWC_AUTO_KEYS: capacity of the per-device auto key cache (default 256 keys, 20 MB of combs
// each, allocated on first use; 0 disables it).
uint32_t auto_keys_cap() {
  static const uint32_t cap = [] {
    const char* e = std::getenv("NWC_AUTO_KEYS");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 256u;
  }();
  return cap;
}
// NWC_COMB16=0: no radix-2^22 basepoint comb at nwc_init (saves 3.2 GB of HBM per device);
// committee batches then take the cached ladder (k_verify<true, true>) instead of the comb
// kernel, and first-sight small calls the one-lane path instead of the cold kernel.
bool comb16_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NWC_COMB16");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

constexpr size_t AUTO_SEEN_MAX = 4096;   // keys remembered as seen once (cleared when full)
constexpr uint32_t AUTO_INIT_KEYS = 16;   // auto-cache capacity allocated at nwc_init (doubled on demand)

// Stream-ordered (re)allocation of the auto cache's arrays to ncap keys: the new arrays come from
// the stream's pool (hipMallocAsync), what is built is copied over, and the old arrays are freed
// behind every launch already queued -- the host never waits.  Caller holds d.mu.
int auto_grow(DevCtx& d, uint32_t ncap) {
  nwc::u32 *keys = nullptr, *flags = nullptr;
  nwc::ge_niels* tables = nullptr;
  nwc::ge_niels_pad* comb = nullptr;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&keys), 32 * (size_t)ncap, d.stream));
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&flags), 4 * (size_t)ncap, d.stream));
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&tables), (size_t)ncap * 129 * sizeof(nwc::ge_niels), d.stream));
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&comb), (size_t)ncap * nwc::COMB_PER_KEY * sizeof(nwc::ge_niels_pad),
                         d.stream));
  const size_t n0 = d.ak_n;
  if (n0) {
    HIP_TRY(hipMemcpyAsync(keys, d.ak_keys, 32 * n0, hipMemcpyDeviceToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(flags, d.ak_flags, 4 * n0, hipMemcpyDeviceToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(tables, d.ak_tables, n0 * 129 * sizeof(nwc::ge_niels), hipMemcpyDeviceToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(comb, d.ak_comb, n0 * nwc::COMB_PER_KEY * sizeof(nwc::ge_niels_pad), hipMemcpyDeviceToDevice,
                           d.stream));
  }
  if (d.ak_keys) HIP_TRY(hipFreeAsync(d.ak_keys, d.stream));
  if (d.ak_flags) HIP_TRY(hipFreeAsync(d.ak_flags, d.stream));
  if (d.ak_tables) HIP_TRY(hipFreeAsync(d.ak_tables, d.stream));
  if (d.ak_comb) HIP_TRY(hipFreeAsync(d.ak_comb, d.stream));
  d.ak_keys = keys; d.ak_flags = flags; d.ak_tables = tables; d.ak_comb = comb;
  d.ak_cap = ncap;
  return 0;
}

// Empties the auto cache (nwc_set_committee: a new committee makes the remembered keys stale).
// The arrays are kept for reuse.  Caller holds d.mu and has drained d.stream.
void auto_reset(DevCtx& d) {
  d.ak_n = 0;
  d.ak_evict = 0;
  d.ak_pending = false;
  d.ak_host = KeyIndex{};
  d.ak_seen.clear();
}

// Keys of a small host call that missed every cache: a key seen before is added to the auto
// cache (flags, 129-entry table and comb built on d.stream after this call's work; the next call
// on this device is ordered after the build), a new one is remembered as seen.  Once the cache
// holds NWC_AUTO_KEYS keys, new ones replace the oldest (FIFO ring): a launch queued before the
// replacement has finished with the old entry when the build runs (one stream), and the host
// index drops the old key at once, so its next call takes the uncached path.  The host copy is
// updated once the build is enqueued; the call does not wait for it (its copy sources stay in
// d.ak_pend_* until the next build has synchronised).  Caller holds d.mu and has set the device.
int auto_insert(DevCtx& d, const uint8_t* pks, uint64_t n) {
  const uint32_t cap = auto_keys_cap();
  if (cap == 0) return 0;
  std::vector<nwc::u32> add;
  std::unordered_set<std::string> added;
  for (uint64_t i = 0; i < n && add.size() / 8 < cap; ++i) {
    const uint8_t* k = pks + 32 * i;
    if (d.ak_host.find(k)) continue;
    std::string ks(reinterpret_cast<const char*>(k), 32);
    if (added.count(ks)) continue;
    if (!d.ak_seen.count(ks)) {
      if (d.ak_seen.size() >= AUTO_SEEN_MAX) d.ak_seen.clear();
      d.ak_seen.insert(std::move(ks));
      continue;
    }
    d.ak_seen.erase(ks);
    added.insert(ks);
    add.insert(add.end(), reinterpret_cast<const nwc::u32*>(k), reinterpret_cast<const nwc::u32*>(k) + 8);
  }
  const uint32_t m = (uint32_t)(add.size() / 8);
  if (m == 0) return 0;
  if (d.ak_pending) {
    HIP_TRY(hipStreamSynchronize(d.stream));   // the previous build's copy sources are free again
    d.ak_pending = false;
  }
  // positions: append while there is room, then the FIFO ring over [0, cap)
  std::vector<uint32_t> pos(m);
  uint32_t n1 = d.ak_n;
  for (uint32_t j = 0; j < m; ++j) {
    if (n1 < cap) {
      pos[j] = n1++;
    } else {
      pos[j] = d.ak_evict;
      d.ak_evict = (d.ak_evict + 1) % cap;
    }
  }
  if (n1 > d.ak_cap)
    if (int rc = auto_grow(d, std::min(cap, std::max<uint32_t>(AUTO_INIT_KEYS, 2 * n1)))) return rc;
  KeyIndex next = d.ak_host;
  next.keys.resize(8 * (size_t)n1);
  for (uint32_t j = 0; j < m; ++j) std::memcpy(&next.keys[8 * (size_t)pos[j]], &add[8 * (size_t)j], 32);
  std::vector<int32_t> table;
  const uint32_t slots = build_slots(next.keys, n1, table);
  if (slots > d.ak_slot_cap) {
    if (d.ak_slots) HIP_TRY(hipFreeAsync(d.ak_slots, d.stream));   // after every launch that reads it
    d.ak_slots = nullptr;
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&d.ak_slots), 4 * (size_t)slots, d.stream));
    d.ak_slot_cap = slots;
  }
  d.ak_pend_keys = std::move(add);
  d.ak_pend_slots = table;
  // contiguous runs of positions (at most two: the appended tail and the ring's start)
  for (uint32_t j0 = 0; j0 < m;) {
    uint32_t j1 = j0 + 1;
    while (j1 < m && pos[j1] == pos[j1 - 1] + 1) ++j1;
    const uint32_t p0 = pos[j0], r = j1 - j0;
    HIP_TRY(hipMemcpyAsync(d.ak_keys + 8 * (size_t)p0, d.ak_pend_keys.data() + 8 * (size_t)j0, 32 * (size_t)r,
                           hipMemcpyHostToDevice, d.stream));
    hipLaunchKernelGGL(nwc::k_build_key_tables, dim3((unsigned)((r * 129 + 255) / 256)), dim3(256), 0, d.stream,
                       d.ak_keys + 8 * (size_t)p0, r, d.ak_tables + (size_t)p0 * 129, d.ak_flags + p0);
    HIP_TRY(hipGetLastError());
    if (int rc = build_key_combs(d, d.ak_keys + 8 * (size_t)p0, r, d.ak_comb + (size_t)p0 * nwc::COMB_PER_KEY)) return rc;
    j0 = j1;
  }
  HIP_TRY(hipMemcpyAsync(d.ak_slots, d.ak_pend_slots.data(), 4 * (size_t)slots, hipMemcpyHostToDevice, d.stream));
  d.ak_pending = true;
  next.slots = std::move(table);
  next.mask = slots - 1;
  d.ak_host = std::move(next);
  d.ak_n = n1;
  ++d.ak_builds;
  return 0;
}

// ---- launch helpers (caller holds the device mutex and has set the device) -----------------
// Verification path (NWC_VERIFY_PATH): default = the doubling-free comb kernel for equations whose
// key is in the committee cache (when the committee has combs) and half-size equations with
// full-length fallback for the rest; "half" = no comb kernel; "full" = the full-length ladder for
// every lane.  The alternatives exist to cross-check the paths against each other.
enum class VPath { Default, Half, Full };
VPath verify_path() {
  static const VPath p = [] {
    const char* e = std::getenv("NWC_VERIFY_PATH");
    if (e && std::strcmp(e, "full") == 0) return VPath::Full;
    if (e && std::strcmp(e, "half") == 0) return VPath::Half;
    return VPath::Default;
  }();
  return p;
}

// Device memory of the verification path (a primary and workers share the GPU:
// worker/src/worker.rs:182,227).  One launch takes at most NWC_VERIFY_MAX_LAUNCH equations (larger
// calls run as consecutive launches of that size, launch_verify), so the per-launch lists below are
// bounded; and lists larger than NWC_VERIFY_KEEP_BYTES are shrunk to a smaller launch's size
// when one comes (after the device has finished with them).  The per-lane table slots are sized
// for the resident grid, not for n.
#ifndef NWC_VERIFY_MAX_LAUNCH
#define NWC_VERIFY_MAX_LAUNCH (16ull << 20)
#endif
uint64_t verify_max_launch() {
  static const uint64_t m = [] {
    const char* e = std::getenv("NWC_VERIFY_MAX_LAUNCH");
    const uint64_t v = e ? std::strtoull(e, nullptr, 10) : (uint64_t)NWC_VERIFY_MAX_LAUNCH;
    return std::max<uint64_t>(1u << 16, v / 64 * 64);
  }();
  return m;
}
size_t verify_keep_bytes() {
  static const size_t k = [] {
    const char* e = std::getenv("NWC_VERIFY_KEEP_BYTES");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)256 << 20;
  }();
  return k;
}
// bytes of the per-launch lists: fb_list, uc_list, ts_uniq (4 B per entry) and the torsion hash set
size_t list_bytes(uint64_t cap, uint64_t slots) { return 12 * (size_t)cap + 8 * (size_t)slots; }
void free_lists(DevCtx& d) {
  for (void* p : {(void*)d.fb_list, (void*)d.uc_list, (void*)d.ts_slots, (void*)d.ts_flag, (void*)d.ts_uniq})
    if (p) (void)hipFree(p);
  d.fb_list = nullptr;
  d.uc_list = nullptr;
  d.ts_slots = nullptr;
  d.ts_flag = nullptr;
  d.ts_uniq = nullptr;
  d.fb_cap = 0;
  d.ts_slot_count = 0;
}

int ensure_scratch(DevCtx& d, size_t bytes, uint64_t n) {
  const uint64_t want = n + n / 2 + 4096;
  const bool shrink = !d.hold_lists && d.fb_cap > 4 * want && list_bytes(d.fb_cap, d.ts_slot_count) > verify_keep_bytes();
  if (bytes <= d.scratch_cap && n <= d.fb_cap && !shrink) return 0;
  HIP_TRY(hipEventSynchronize(d.scratch_free));
  if (bytes > d.scratch_cap) {
    if (d.scratch) HIP_TRY(hipFree(d.scratch));
    d.scratch = nullptr;
    d.scratch_cap = 0;
    HIP_TRY(hipMalloc(&d.scratch, bytes));
    d.scratch_cap = bytes;
  }
  if (shrink || n > d.fb_cap) {
    free_lists(d);
    const size_t c = want;
    HIP_TRY(hipMalloc(&d.fb_list, 4 * c));
    HIP_TRY(hipMalloc(&d.uc_list, 4 * c));
    // the hash set stays at most half full: >= 2 slots per equation
    uint32_t slots = 1024;
    while (slots < 2 * c) slots <<= 1;
    HIP_TRY(hipMalloc(&d.ts_slots, 4 * (size_t)slots));
    HIP_TRY(hipMalloc(&d.ts_flag, 4 * (size_t)slots));
    HIP_TRY(hipMalloc(&d.ts_uniq, 4 * c));
    d.ts_slot_count = slots;
    d.fb_cap = c;
  }
  if (!d.ts_nuniq) HIP_TRY(hipMalloc(&d.ts_nuniq, sizeof(uint32_t)));
  return 0;
}

// Batch-leaf launches: clear the verdict bits of equations whose key has an 8-torsion component
// (dalek verify_batch's randomized domain, answered Err; kernels.hip k_tors_*).  list/count
// (device) restrict the pass to the comb path's uncached equations; nullptr = all n.  The hash set
// is sized for the number of candidate equations, which never exceeds n <= fb_cap.
// phase 1 = mark + eval, 2 = apply, 3 = both.  pre: phase 1 runs before or beside the
// verification (every equation a candidate; the verdict words untouched until apply).
int launch_torsion(DevCtx& d, const uint8_t* pks, uint64_t* out_words, uint64_t n, const uint32_t* list,
                   const uint32_t* count, const nwc::Committee& cm, hipStream_t s, int phase = 3, int pre = 0) {
  if (n == 0) return 0;
  if (2 * n > d.ts_slot_count) return set_err(NWC_ERR_ARG, "torsion set too small for %llu equations", (unsigned long long)n);
  const nwc::KeyMemo memo{d.km_keys, d.km_flag, NWC_MEMO_SLOTS - 1};
  const nwc::TorsArgs t{pks, out_words, list, count, n, d.ts_slots, d.ts_slot_count - 1, d.ts_uniq, d.ts_nuniq, d.ts_flag, cm,
                        memo, pre};
  const uint64_t cap = (uint64_t)d.cus * 8;
  const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, cap);
  if (phase & 1) {
    HIP_TRY(hipMemsetAsync(d.ts_slots, 0xFF, 4 * (size_t)d.ts_slot_count, s));
    HIP_TRY(hipMemsetAsync(d.ts_nuniq, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(nwc::k_tors_mark, dim3(grid), dim3(256), 0, s, t);
    HIP_TRY(hipGetLastError());
    if (n <= NWC_WIDE_MAX) {
      // a certificate's worth of keys: one limb-sliced wave per distinct key (latency)
      hipLaunchKernelGGL(nwc::k_tors_eval_sliced, dim3((unsigned)n), dim3(64), 0, s, t);
    } else {
      hipLaunchKernelGGL(nwc::k_tors_eval, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, (uint64_t)d.cus * 2)), dim3(256), 0, s, t);
    }
    HIP_TRY(hipGetLastError());
  }
  if (phase & 2) {
    hipLaunchKernelGGL(nwc::k_tors_apply, dim3(grid), dim3(256), 0, s, t);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

// NWC_COLD=0: small uncached calls take k_verify (one lane per equation) instead of the
// limb-sliced k_verify_cold (A/B and tests)
bool cold_path() {
  static const bool on = [] {
    const char* e = std::getenv("NWC_COLD");
    return !(e && std::strcmp(e, "0") == 0) && comb16_enabled();   // its s B is a comb16 sum
  }();
  return on;
}

// largest launch the cold kernel takes (one 4-wave block per equation); above it the one-lane
// ladder's throughput wins (tools/cold_sizes.py)
#ifndef NWC_COLD_MAX
#define NWC_COLD_MAX 3072
#endif
uint64_t cold_max() {
  static const uint64_t m = [] {
    const char* e = std::getenv("NWC_COLD_MAX");   // A/B
    return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)NWC_COLD_MAX;
  }();
  return m;
}

// Device buffers of the launch keys (launch_keys.h), allocated once per device except the combs
// (20 MB per key), which grow as keys ask to join; the set starts empty.  Caller holds d.mu.
int lk_ensure(DevCtx& d, hipStream_t s) {
  if (d.lk_alloc) return 0;
  nwc::LaunchKeys& k = d.lk;
  HIP_TRY(hipMalloc(&k.keys, 32 * (size_t)nwc::LK_MAX_KEYS));
  HIP_TRY(hipMalloc(&k.flags, 4 * (size_t)nwc::LK_MAX_KEYS));
  HIP_TRY(hipMalloc(&k.slots, 4 * (size_t)nwc::LK_SLOTS));
  HIP_TRY(hipMalloc(&k.bases, (size_t)nwc::LK_MAX_KEYS * nwc::KeyComb::windows * sizeof(nwc::ge_p3)));
  HIP_TRY(hipMalloc(&k.state, 16));
  if (!d.lk_demand) HIP_TRY(hipHostMalloc(&d.lk_demand, sizeof(uint32_t), hipHostMallocCoherent));
  {
    // (again after nwc_trim, which resets the set's struct but keeps this word)
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, d.lk_demand, 0));
    k.host_demand = static_cast<uint32_t*>(dp);
  }
  *reinterpret_cast<volatile uint32_t*>(d.lk_demand) = 0;
  k.comb = nullptr;
  k.cap = 0;
  HIP_TRY(hipMemsetAsync(k.slots, 0xFF, 4 * (size_t)nwc::LK_SLOTS, s));
  HIP_TRY(hipMemsetAsync(k.state, 0, 16, s));
  d.lk_alloc = true;
  d.lk_censused = false;
  return 0;
}

// Room for the keys that asked to join: the first launch-key launch (and the first after
// nwc_set_committee emptied the set) runs the census once and waits for its demand; later launches
// read the demand the previous ones left in host memory (no sync) and grow the combs
// stream-ordered on s (held combs copied), so a key that did not fit joins at the next launch.
// Called after s waits for scratch_free (no launch still reads the set).
int lk_reserve(DevCtx& d, const uint8_t* pks, uint64_t n, hipStream_t s) {
  nwc::LaunchKeys& k = d.lk;
  if (k.cap >= nwc::LK_MAX_KEYS) return 0;
  if (!d.lk_censused) {
    // nothing held: with the room for no key the select only counts, then the host reads its demand
    nwc::LaunchKeys count_only = k;
    count_only.cap = 0;
    hipLaunchKernelGGL(nwc::k_lk_select, dim3(1), dim3(1024), 0, s, pks, n, count_only);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    d.lk_censused = true;
  }
  const uint32_t demand = *reinterpret_cast<volatile uint32_t*>(d.lk_demand);
  if (demand <= k.cap) return 0;
  const uint32_t cap = std::min<uint32_t>(nwc::LK_MAX_KEYS, (demand + 7) / 8 * 8);
  nwc::ge_niels_pad* comb = nullptr;
  const size_t per = nwc::COMB_PER_KEY * sizeof(nwc::ge_niels_pad);
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&comb), (size_t)cap * per, s));
  if (k.comb) {
    HIP_TRY(hipMemcpyAsync(comb, k.comb, (size_t)k.cap * per, hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipFreeAsync(k.comb, s));
  }
  k.comb = comb;
  k.cap = cap;
  return 0;
}

// Large host calls copy their pageable inputs through the device's pinned stages, filled by
// NWC_HOST_STAGING_THREADS (8) host threads (straight from pageable memory measured 7-10 % slower,
// profiles/r05/wire_host.md; that switch was removed in round 6).
// NWC_HOST_TIMING: per-phase times of large host calls on stderr (diagnostics)
bool host_timing() {
  static const bool on = std::getenv("NWC_HOST_TIMING") != nullptr;
  return on;
}
unsigned stager_threads() {
  static const unsigned t = [] {
    const char* e = std::getenv("NWC_HOST_STAGING_THREADS");
    return e ? (unsigned)std::max(1, std::atoi(e)) : 8u;
  }();
  return t;
}

// The device's transfer stream and its pinned stages.  Caller holds d.mu.
int ensure_stager(DevCtx& d) {
  if (!d.xfer) HIP_TRY(hipStreamCreateWithFlags(&d.xfer, hipStreamNonBlocking));
  if (!d.stager) {
    auto st = std::make_unique<HostStager>();
    const hipError_t e = st->init(d.xfer, stager_threads());
    if (e != hipSuccess) {
      st->release();
      return set_err(NWC_ERR_DEVICE, "host stager: %s", hipGetErrorString(e));
    }
    d.stager = std::move(st);
  }
  return 0;
}

// The batch entries' buffers (Straus tables, MSM groups, the per-certificate resolution) above
// NWC_VERIFY_KEEP_BYTES that the current launch does not use are freed -- after every launch that
// used them, each of which records scratch_free -- so a process that ran the Straus or MSM entry
// once holds at most the keep threshold of them while it verifies by other paths.
int release_idle_buffers(DevCtx& d, const uint8_t* in_use) {
  const size_t keep = verify_keep_bytes();
  struct Buf { uint8_t** p; size_t* cap; } bufs[] = {
      {&d.straus_scratch, &d.straus_cap}, {&d.msm_scratch, &d.msm_cap}, {&d.rs_buf, &d.rs_cap},
      {&d.pair_buf, &d.pair_cap}, {&d.sign_buf, &d.sign_cap}};
  auto idle = [&](const Buf& b) { return *b.p && *b.p != in_use && *b.p != d.busy_buf && *b.cap > keep; };
  bool any = false;
  for (const Buf& b : bufs) any = any || idle(b);
  if (!any) return 0;
  HIP_TRY(hipEventSynchronize(d.scratch_free));
  for (const Buf& b : bufs) {
    if (idle(b)) {
      HIP_TRY(hipFree(*b.p));
      *b.p = nullptr;
      *b.cap = 0;
    }
  }
  return 0;
}

// launch_verify flags: the caller checked on the host that every key is in the committee cache,
// and/or out_words is already zero (both let the latency path run as a single kernel)
// LV_AUTO: the keys are in the auto cache; LV_STAMP: the headline kernel's clock-stamp build
// (k_verify<.., STAMP>, nwc_diag_verify_clock)
// LV_DEFER_LIST: a launch on the committee-cache comb path (deferrable_list()) that only appends
// its uncached equations, as list_base + i, to the call-wide list; the caller zeroed the list's
// count and sized the lists (ensure_scratch) for the whole call before the first such launch, and
// runs the list, fallback and torsion passes once over all of them (finish_deferred_list).  The
// chunked sanitize pipeline: one set of those small launches per call instead of per chunk.
constexpr int LV_ALL_CACHED = 1, LV_OUT_ZEROED = 2, LV_AUTO = 4, LV_STAMP = 8, LV_DEFER_LIST = 16;

// One launch of the paired strict host pipeline (verify_range): launches on two streams may run at
// the same time, so each takes half of the table slots (`half`; grid capped at half the persistent
// grid) and lists its failed reductions in its own region of the fallback list with its own count;
// the caller orders the slots against other launches (scratch_free), sized the list beforehand and
// runs the fallback passes once the pipeline has joined (a fallback launch queued behind a chunk
// would wait for free slots while the other stream's chunk holds them, stalling its stream).
struct PairLaunch {
  int half;
  uint32_t* fb_list;
  uint32_t* fb_count;
};

// launch_verify's comb path over the committee cache for any n (what LV_DEFER_LIST needs)
bool deferrable_list(const DevCtx& d) {
  return verify_path() == VPath::Default && d.cm_n && d.cm_comb && d.comb16;
}

// NWC_FORCE_FALLBACK_EVERY: test hook, every k-th equation of the half-size kernels takes the fallback
uint32_t force_fallback_every() {
  static const uint32_t v = [] {
    const char* e = std::getenv("NWC_FORCE_FALLBACK_EVERY");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
  }();
  return v;
}

int launch_verify(DevCtx& d, const uint8_t* msgs, const uint32_t* msg_index, uint64_t msg_stride,
                  const uint8_t* pks, const uint8_t* sigs, uint64_t n, int strict, uint64_t* out_words,
                  hipStream_t s, int flags = 0, uint8_t* vbytes = nullptr, uint64_t list_base = 0,
                  const PairLaunch* pl = nullptr, const nwc::SignRecs* sr = nullptr,
                  const nwc::SignPass* sp = nullptr) {
  if (n == 0) return 0;
  if (int rc = ensure_verify_tables(d)) return rc;
  if (int rc = release_idle_buffers(d, nullptr)) return rc;
  if (n > verify_max_launch() && !vbytes) {
    // consecutive launches of at most NWC_VERIFY_MAX_LAUNCH equations (a multiple of 64: whole
    // verdict words), so the per-launch lists stay bounded; every equation is independent, so the
    // verdicts are those of one launch (launch keys and the torsion set are per launch anyway)
    const uint64_t step = verify_max_launch();
    for (uint64_t lo = 0; lo < n; lo += step) {
      const uint64_t len = std::min(step, n - lo);
      if (int rc = launch_verify(d, msg_index ? msgs : msgs + 32 * lo * msg_stride, msg_index ? msg_index + lo : nullptr,
                                 msg_stride, pks + 32 * lo, sigs + 64 * lo, len, strict, out_words + lo / 64, s, flags,
                                 nullptr, list_base + lo))
        return rc;
    }
    return 0;
  }
  // equation indices travel as uint32 (fallback / uncached / torsion lists)
  if (n > 0xFFFFFFFFull) return set_err(NWC_ERR_ARG, "more than 2^32 - 1 equations in one launch");
  const VPath path = verify_path();
  if ((flags & LV_AUTO) && (flags & LV_ALL_CACHED) && path == VPath::Default && n <= NWC_WIDE_MAX && d.ak_n) {
    // latency path over the auto key cache (same kernel, the auto cache as its committee)
    ++d.ak_hits;
    const nwc::Committee cm{d.ak_keys, d.ak_flags, d.ak_tables, d.ak_comb, d.ak_slots, d.ak_host.mask, d.ak_n};
    const nwc::VerifyArgs a{msgs, msg_index, msg_stride, pks, sigs, out_words, n, strict, d.base_table, d.base24,
                            d.scratch, d.fb_list, d.fb_count, 0u, cm};
    const nwc::CombArgs ca{nullptr, reinterpret_cast<uint32_t*>(out_words + (n + 63) / 64), d.comb_base, d.comb16,
                           vbytes};
    if (!vbytes && !(flags & LV_OUT_ZEROED)) HIP_TRY(hipMemsetAsync(out_words, 0, 8 * ((n + 63) / 64 + 1), s));
    hipLaunchKernelGGL(nwc::k_verify_comb_wide, dim3((unsigned)n), dim3(128), 0, s, a, ca);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  const uint32_t force_every = force_fallback_every();
  if (vbytes && !(flags & LV_ALL_CACHED)) {
    // zero-copy cold launch (the caller checked: no committee cache, n <= NWC_WIDE_MAX, default
    // path, cold kernel on): no scratch, no fallback launch, verdict bytes straight to the host
    const nwc::VerifyArgs a{msgs, msg_index, msg_stride, pks, sigs, out_words, n, strict, d.base_table, d.base24,
                            d.scratch, d.fb_list, d.fb_count, force_every, nwc::Committee{}};
    hipLaunchKernelGGL(nwc::k_verify_cold, dim3((unsigned)n), dim3(256), 0, s, a, (const nwc::ge_niels_pad*)d.comb16, vbytes);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  // (the throughput comb kernel needs the basepoint comb16; the latency kernel does not)
  // A large batch-leaf launch without a committee cache brings its own committee: the keys it
  // repeats join the launch-key set and its votes take the comb kernel (launch_keys.h).
  const bool lk = path == VPath::Default && !strict && !d.cm_n && d.comb16 && n >= nwc::LK_MIN_EQUATIONS &&
                  knobs().launch_keys.load() && !(flags & LV_AUTO);
  const bool comb = lk || (path == VPath::Default && d.cm_n && d.cm_comb && (n <= NWC_WIDE_MAX || d.comb16));
  const bool defer = (flags & LV_DEFER_LIST) != 0;
  if (defer && (lk || !comb || list_base + n > d.fb_cap || !deferrable_list(d)))
    return set_err(NWC_ERR_ARG, "deferred list launch off the committee-cache comb path");
  if (sr && (!comb || (defer && (list_base & 63))))
    return set_err(NWC_ERR_ARG, "sign-deferred launch off the comb path or off a verdict word");
  if (comb && n <= NWC_WIDE_MAX && (flags & LV_ALL_CACHED)) {
    // latency path, one launch: no scratch, no uncached list, no fallback (the comb path has none).
    // The host checked every key against its view of the cache (set under g_cm_mu, like the
    // devices'); should a key still be missing on the device, the kernel sets the word after the
    // verdict words instead of listing it, and the caller re-runs the general path.
    const nwc::Committee cm{d.cm_keys, d.cm_flags, d.cm_tables, d.cm_comb, d.cm_slots, d.cm_slot_mask, d.cm_n};
    const nwc::VerifyArgs a{msgs, msg_index, msg_stride, pks, sigs, out_words, n, strict, d.base_table, d.base24,
                            d.scratch, d.fb_list, d.fb_count, 0u, cm};
    const nwc::CombArgs ca{nullptr, reinterpret_cast<uint32_t*>(out_words + (n + 63) / 64), d.comb_base, d.comb16,
                           vbytes};
    if (!vbytes && !(flags & LV_OUT_ZEROED)) HIP_TRY(hipMemsetAsync(out_words, 0, 8 * ((n + 63) / 64 + 1), s));
    hipLaunchKernelGGL(nwc::k_verify_comb_wide, dim3((unsigned)n), dim3(128), 0, s, a, ca);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  const uint64_t tiles = (n + 255) / 256;
  // persistent grid: a few blocks per resident slot so the tail is short
  const uint64_t cap = (uint64_t)d.cus * d.verify_blocks_per_cu * NWC_VERIFY_GRID_MULT;
  size_t need = (size_t)cap * 256 * 2 * nwc::TAB_BYTES_PER_LANE;
  const bool pair = pl != nullptr;
  const uint64_t gcap = pair ? cap / 2 : cap;
  const unsigned grid = (unsigned)(tiles < gcap ? tiles : gcap);
  // comb grid: at most the resident blocks; tile t goes to block t mod grid, so every lane gets
  // ceil or floor of n / lanes equations (in chunks of COMB_BATCH sharing one inversion), and
  // a small n spreads one equation per lane
  unsigned gridc = 0;
  if (comb) {
    const uint64_t resident = (uint64_t)d.cus * d.comb_blocks_per_cu;
    gridc = (unsigned)std::min<uint64_t>(tiles, resident);
    need = std::max(need, (size_t)resident * 256 * nwc::COMB_BYTES_PER_LANE);
  }
  // (deferred: n = the lists' capacity, so they are neither grown nor shrunk under the pending list)
  if (int rc = ensure_scratch(d, need, defer ? d.fb_cap : n)) return rc;
  if (lk)
    if (int rc = lk_ensure(d, s)) return rc;
  if (pair && (!strict || comb || path == VPath::Full || d.cm_n))
    return set_err(NWC_ERR_ARG, "paired launch off the strict half-size path");
  if (!pair) HIP_TRY(hipStreamWaitEvent(s, d.scratch_free, 0));
  if (lk) {
    // the set's update is ordered after every launch that read it (scratch_free) and before this
    // launch's comb kernel; the builds exit at once when no key joined
    if (int rc = lk_reserve(d, pks, n, s)) return rc;
    hipLaunchKernelGGL(nwc::k_lk_select, dim3(1), dim3(1024), 0, s, pks, n, d.lk);
    hipLaunchKernelGGL(nwc::k_lk_keys, dim3((nwc::LK_MAX_KEYS + 63) / 64), dim3(64), 0, s, d.lk);
    hipLaunchKernelGGL(nwc::k_build_comb_from_bases<nwc::KeyComb>, dim3((unsigned)(d.cus * 8)), dim3(256), 0, s,
                       (const nwc::ge_p3*)d.lk.bases, 0u, 0u, (const uint32_t*)d.lk.state, d.lk.comb);
    HIP_TRY(hipGetLastError());
  }
  const nwc::Committee cm = lk ? nwc::Committee{d.lk.keys, d.lk.flags, nullptr, d.lk.comb, d.lk.slots, nwc::LK_SLOTS - 1,
                                                nwc::LK_MAX_KEYS}
                               : nwc::Committee{d.cm_keys, d.cm_flags, d.cm_tables, d.cm_comb, d.cm_slots, d.cm_slot_mask, d.cm_n};
  nwc::VerifyArgs a{msgs, msg_index, msg_stride, pks, sigs, out_words, n, strict, d.base_table, d.base24, d.scratch,
                    d.fb_list, d.fb_count, force_every, cm};
  if (pair) {
    a.scratch = d.scratch + (size_t)(pl->half ? cap / 2 : 0) * 256 * 2 * nwc::TAB_BYTES_PER_LANE;
    a.fb_list = pl->fb_list;
    a.fb_count = pl->fb_count;
  }
  a.force_windows = knobs().force_windows.load();
  a.stamps = d.stamps;
  const nwc::CombArgs ca{d.uc_list, d.uc_count, d.comb_base, d.comb16, nullptr, (uint32_t)(defer ? list_base : 0)};
  const bool half = path != VPath::Full;
  // small batch-leaf launches outside the comb path: the keys' torsion test (one long serial
  // lane per new key) runs on the side stream beside the verification instead of after it
  // a small batch no cache covers (first-sight keys): one limb-sliced block per equation, the
  // batch leaf's torsion test inside it
  const bool cold = half && !comb && !cm.n && n <= cold_max() && cold_path() && !pair;
  const bool tors_beside = !strict && !comb && n <= NWC_WIDE_MAX && !cold;
  if (tors_beside) {
    HIP_TRY(hipEventRecord(d.ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(d.side, d.ev_fork, 0));
    if (int rc = launch_torsion(d, pks, out_words, n, nullptr, nullptr, cm, d.side, 1, 1)) return rc;
    HIP_TRY(hipEventRecord(d.ev_join, d.side));
  }
  if (defer && sr) {
    // R' and the projective y test now, the sign of x(R') later in k_comb_sign over many votes
    // (or in the first blocks of the next such launch: sp, the previous launch's votes)
    const unsigned gy = (unsigned)std::min<uint64_t>(tiles, 60000);
    if (sp && sp->n)
      hipLaunchKernelGGL(nwc::k_verify_comb_y_sign, dim3(gy + sp->blocks), dim3(256), 0, s, a, ca, *sr, *sp);
    else
      hipLaunchKernelGGL(nwc::k_verify_comb_y, dim3(gy), dim3(256), 0, s, a, ca, *sr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(d.scratch_free, s));
    return 0;
  }
  if (defer) {
    if (n <= NWC_WIDE_MAX) {
      HIP_TRY(hipMemsetAsync(out_words, 0, 8 * ((n + 63) / 64), s));
      hipLaunchKernelGGL(nwc::k_verify_comb_wide, dim3((unsigned)n), dim3(128), 0, s, a, ca);
    } else {
      hipLaunchKernelGGL(nwc::k_verify_comb, dim3(gridc), dim3(256), 0, s, a, ca);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(d.scratch_free, s));
    return 0;
  }
  if (half) HIP_TRY(hipMemsetAsync(a.fb_count, 0, sizeof(uint32_t), s));
  if (comb) {
    HIP_TRY(hipMemsetAsync(d.uc_count, 0, sizeof(uint32_t), s));
    if (sr) {
      // sign test deferred (the chunked host path, verify_range): the words zeroed for the list
      // passes and the later sign pass to OR into; the previous chunk's sign pass in front
      HIP_TRY(hipMemsetAsync(out_words, 0, 8 * ((n + 63) / 64), s));
      const unsigned gy = (unsigned)std::min<uint64_t>(tiles, 60000);
      if (sp && sp->n)
        hipLaunchKernelGGL(nwc::k_verify_comb_y_sign, dim3(gy + sp->blocks), dim3(256), 0, s, a, ca, *sr, *sp);
      else
        hipLaunchKernelGGL(nwc::k_verify_comb_y, dim3(gy), dim3(256), 0, s, a, ca, *sr);
    } else if (n <= NWC_WIDE_MAX) {
      // small batches: one block per equation, critical path = one square root
      HIP_TRY(hipMemsetAsync(out_words, 0, 8 * ((n + 63) / 64), s));
      hipLaunchKernelGGL(nwc::k_verify_comb_wide, dim3((unsigned)n), dim3(128), 0, s, a, ca);
    } else {
      hipLaunchKernelGGL(nwc::k_verify_comb, dim3(gridc), dim3(256), 0, s, a, ca);
    }
    HIP_TRY(hipGetLastError());
    // uncached keys: half-size equations in list mode (waves exit at once when the list is empty)
    nwc::VerifyArgs l = a;
    l.committee.n = 0;
    hipLaunchKernelGGL((nwc::k_verify<true, false, true>), dim3(grid), dim3(256), 0, s, l, ca);
  } else if (cold) {
    if (!(flags & LV_OUT_ZEROED)) HIP_TRY(hipMemsetAsync(out_words, 0, 8 * ((n + 63) / 64), s));
    hipLaunchKernelGGL(nwc::k_verify_cold, dim3((unsigned)n), dim3(256), 0, s, a, (const nwc::ge_niels_pad*)d.comb16,
                       (uint8_t*)nullptr);
  } else {
    if (half && cm.n)
      hipLaunchKernelGGL((nwc::k_verify<true, true>), dim3(grid), dim3(256), 0, s, a, ca);
    else if (half && (flags & LV_STAMP))
      hipLaunchKernelGGL((nwc::k_verify<true, false, false, true>), dim3(grid), dim3(256), 0, s, a, ca);
    else if (half)
      hipLaunchKernelGGL((nwc::k_verify<true, false>), dim3(grid), dim3(256), 0, s, a, ca);
    else
      hipLaunchKernelGGL((nwc::k_verify<false, false>), dim3(grid), dim3(256), 0, s, a, ca);
  }
  HIP_TRY(hipGetLastError());
  if (half && !pair) {
    // lanes whose reduction failed are rare (|c| or d >= 2^147); a few blocks suffice
    const unsigned fgrid = grid < 16u ? grid : 16u;
    hipLaunchKernelGGL(nwc::k_verify_fallback, dim3(fgrid), dim3(256), 0, s, a);
    HIP_TRY(hipGetLastError());
  }
  // batch leaves: keys with torsion (cached keys were checked in the comb kernels; the comb
  // path's other equations are its uncached list)
  if (tors_beside) {
    HIP_TRY(hipStreamWaitEvent(s, d.ev_join, 0));
    if (int rc = launch_torsion(d, pks, out_words, n, nullptr, nullptr, cm, s, 2, 1)) return rc;
  } else if (!strict && !cold) {
    if (int rc = launch_torsion(d, pks, out_words, n, comb ? d.uc_list : nullptr, comb ? d.uc_count : nullptr, cm, s))
      return rc;
  }
  if (!pair) HIP_TRY(hipEventRecord(d.scratch_free, s));
  return 0;
}

// The passes LV_DEFER_LIST launches left out, once over equations [0, n) of the arrays they were
// launched on (their list holds indices into these): the uncached equations' half-size list
// launch, its fallback and (batch leaves) the torsion pass over the same list.
int finish_deferred_list(DevCtx& d, const uint8_t* msgs, const uint32_t* msg_index, uint64_t msg_stride,
                         const uint8_t* pks, const uint8_t* sigs, uint64_t n, int strict, uint64_t* out_words,
                         hipStream_t s) {
  if (n == 0) return 0;
  if (!deferrable_list(d) || n > d.fb_cap) return set_err(NWC_ERR_ARG, "deferred list finish off the comb path");
  const uint64_t tiles = (n + 255) / 256;
  const uint64_t cap = (uint64_t)d.cus * d.verify_blocks_per_cu * NWC_VERIFY_GRID_MULT;
  const unsigned grid = (unsigned)(tiles < cap ? tiles : cap);
  if (int rc = ensure_scratch(d, (size_t)cap * 256 * 2 * nwc::TAB_BYTES_PER_LANE, d.fb_cap)) return rc;
  HIP_TRY(hipStreamWaitEvent(s, d.scratch_free, 0));
  const nwc::Committee cm{d.cm_keys, d.cm_flags, d.cm_tables, d.cm_comb, d.cm_slots, d.cm_slot_mask, d.cm_n};
  nwc::VerifyArgs a{msgs, msg_index, msg_stride, pks, sigs, out_words, n, strict, d.base_table, d.base24, d.scratch,
                    d.fb_list, d.fb_count, force_fallback_every(), cm};
  a.force_windows = knobs().force_windows.load();
  a.stamps = d.stamps;
  const nwc::CombArgs ca{d.uc_list, d.uc_count, d.comb_base, d.comb16};
  HIP_TRY(hipMemsetAsync(d.fb_count, 0, sizeof(uint32_t), s));
  nwc::VerifyArgs l = a;
  l.committee.n = 0;
  hipLaunchKernelGGL((nwc::k_verify<true, false, true>), dim3(grid), dim3(256), 0, s, l, ca);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(nwc::k_verify_fallback, dim3(grid < 16u ? grid : 16u), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  if (!strict)
    if (int rc = launch_torsion(d, pks, out_words, n, d.uc_list, d.uc_count, cm, s)) return rc;
  HIP_TRY(hipEventRecord(d.scratch_free, s));
  return 0;
}

// sr with its arrays moved by `off` records (record i of the result is record i + off of sr)
nwc::SignRecs sign_recs_at(const nwc::SignRecs& r, int64_t off) {
  return nwc::SignRecs{r.x + 8 * off, r.z + 8 * off, r.p + 8 * off, r.meta + off};
}
// k_comb_sign over votes [v0, v0 + n) of sr (v0 a multiple of 64): about 8 votes per lane, so the
// lane's one inversion is shared, and at most the resident comb lanes
uint32_t comb_sign_blocks(const DevCtx& d, uint64_t n) {
  constexpr uint64_t per = 8;   // votes per lane
  const uint64_t resident = (uint64_t)d.cus * d.comb_blocks_per_cu;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(resident, (n + 256 * per - 1) / (256 * per)));
}
int launch_comb_sign(DevCtx& d, const nwc::SignRecs& sr, uint64_t v0, uint64_t n, uint64_t* out_bits, hipStream_t s) {
  if (n == 0) return 0;
  if (v0 & 63) return set_err(NWC_ERR_ARG, "sign pass off a verdict word");
  const uint32_t blocks = comb_sign_blocks(d, n);
  hipLaunchKernelGGL(nwc::k_comb_sign, dim3(blocks), dim3(256), 0, s, sr, v0, n, out_bits);
  HIP_TRY(hipGetLastError());
  return 0;
}

// NWC_SIGN_DEFER=0: the comb path decides the sign in k_verify_comb everywhere (A/B of the
// deferred sign tests of chunked launches: the message pipeline and large host calls)
bool sign_defer() {
  static const bool on = [] {
    const char* e = std::getenv("NWC_SIGN_DEFER");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}
// NWC_STRICT_Y=0: the message pipeline's strict equations through launch_verify on the leaf
// stream (A/B of the list-free strict launches on the parse stream)
bool strict_y_on() {
  static const bool on = [] {
    const char* e = std::getenv("NWC_STRICT_Y");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}
// Whether launch_verify takes the comb path (k_verify_comb) for a plain launch of n equations.
bool takes_comb_path(const DevCtx& d, uint64_t n, int strict) {
  if (verify_path() != VPath::Default) return false;
  const bool lk = !strict && !d.cm_n && d.comb16 && n >= nwc::LK_MIN_EQUATIONS && knobs().launch_keys.load();
  return lk || (d.cm_n && d.cm_comb && (n <= NWC_WIDE_MAX || d.comb16));
}
// NWC_DIGEST_SCHED=0/1 forces the one-lane-per-message / scheduled digest kernel (A/B and tests).
int digest_sched_mode() {
  static const int mode = [] {
    const char* e = std::getenv("NWC_DIGEST_SCHED");
    return e ? std::atoi(e) : -1;
  }();
  return mode;
}

int launch_digest(const uint8_t* data, const uint64_t* offsets, const uint64_t* ends, uint64_t n, uint8_t* out32,
                  hipStream_t s) {
  if (n == 0) return 0;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  int cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // more than one wave per SIMD of one-lane-per-message work: schedule blocks instead
  const int mode = digest_sched_mode();
  const bool sched = mode >= 0 ? mode == 1 : n > 64ull * 4 * (uint64_t)cus;
  if (sched) {
    hipLaunchKernelGGL(nwc::k_sha512_digest32_sched, dim3((unsigned)cus), dim3(256), 0, s, data, offsets, ends, n,
                       out32);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(nwc::k_sha512_digest32, dim3(grid), dim3(256), 0, s, data, offsets, ends, n, out32);
  HIP_TRY(hipGetLastError());
  return 0;
}

int launch_cert_reduce(const uint64_t* leaf, const uint32_t* offs, uint64_t m, uint64_t nvotes, uint64_t* cert,
                       uint64_t* bad, hipStream_t s) {
  const uint64_t words = (nvotes + 63) / 64;
  const uint64_t threads = m > words ? m : words;
  if (threads == 0) return 0;
  const unsigned grid = (unsigned)((threads + 255) / 256);
  hipLaunchKernelGGL(nwc::k_cert_reduce, dim3(grid), dim3(256), 0, s, leaf, offs, m, nvotes, cert, bad);
  HIP_TRY(hipGetLastError());
  return 0;
}

// Run fn(device_index, lo, hi) over [0, n) split across all devices, one host thread each.  The
// ranges come from nwc_shard_bounds: every range but the last starts on a multiple of 64 units.
template <class F>
int shard(uint64_t n, F fn) {
  const int nd = (int)g_devs.size();
  if (nd == 1 || n < 4096) return fn(0, (uint64_t)0, n);
  std::vector<int> rc(nd, 0);
  std::vector<std::thread> th;
  for (int i = 0; i < nd; ++i) {
    uint64_t lo = 0, hi = 0;
    nwc_shard_bounds(n, (uint32_t)nd, (uint32_t)i, &lo, &hi);
    th.emplace_back([&, i, lo, hi] {
      rc[i] = fn(i, lo, hi);
    });
  }
  for (auto& t : th) t.join();
  for (int r : rc) if (r < 0) return r;
  return 0;
}

// Copy `nbits` bits of device verdict words to a host bitmap starting at bit `bit0`.
void merge_bits(uint8_t* dst, uint64_t bit0, const std::vector<uint64_t>& words, uint64_t nbits) {
  // dst bits [bit0, bit0 + nbits) = source bits [0, nbits); bits of dst outside the range kept
  auto put1 = [&](uint64_t b) {
    const uint64_t o = bit0 + b;
    const bool v = (words[b >> 6] >> (b & 63)) & 1;
    dst[o >> 3] = (uint8_t)((dst[o >> 3] & ~(1u << (o & 7))) | ((unsigned)v << (o & 7)));
  };
  uint64_t b = 0;
  if ((bit0 & 7) == 0) {
    const uint64_t full = nbits / 8;
    std::memcpy(dst + bit0 / 8, words.data(), full);
    b = full * 8;
  } else {
    // head bits up to a destination byte boundary, then 8 source bits per destination byte
    for (; b < nbits && ((bit0 + b) & 7); ++b) put1(b);
    for (; b + 8 <= nbits; b += 8) {
      const uint64_t w = b >> 6, sh = b & 63;
      uint64_t v = words[w] >> sh;
      if (sh > 56 && w + 1 < words.size()) v |= words[w + 1] << (64 - sh);
      dst[(bit0 + b) >> 3] = (uint8_t)v;
    }
  }
  for (; b < nbits; ++b) put1(b);
}

// Certificates [c_lo, c_end) of offsets (m + 1 entries) whose votes meet [lo, hi), lo < hi <= offsets[m].
void cert_span(const uint32_t* offsets, uint64_t m, uint64_t lo, uint64_t hi, uint64_t& c_lo, uint64_t& c_end) {
  c_lo = (uint64_t)(std::upper_bound(offsets, offsets + m + 1, (uint32_t)lo) - offsets) - 1;   // offsets[c_lo] <= lo
  c_end = (uint64_t)(std::lower_bound(offsets, offsets + m + 1, (uint32_t)hi) - offsets);     // first offsets[c] >= hi
}

// vote -> certificate index of votes [lo, hi) on the host (small calls; k_cert_index on the device)
void fill_cert_index(uint32_t* dst, const uint32_t* offsets, uint64_t c_lo, uint64_t c_end, uint64_t lo, uint64_t hi) {
  for (uint64_t c = c_lo; c < c_end; ++c) {
    const uint64_t a = std::max<uint64_t>(offsets[c], lo), b = std::min<uint64_t>(offsets[c + 1], hi);
    if (b > a) std::fill(dst + (a - lo), dst + (b - lo), (uint32_t)c);
  }
}

// vote -> certificate index of votes [lo, hi) on stream s, from the offsets already at doffs
// (certificates c_lo .. c_end)
void launch_cert_index(const uint32_t* doffs, uint64_t c_lo, uint64_t c_end, uint64_t lo, uint64_t hi, uint32_t* dmi,
                       hipStream_t s) {
  const uint64_t ncert = c_end - c_lo;
  const unsigned grid = (unsigned)std::min<uint64_t>((ncert * 64 + 255) / 256, 16384);
  hipLaunchKernelGGL(nwc::k_cert_index, dim3(grid), dim3(256), 0, s, doffs, (uint32_t)c_lo, (uint32_t)ncert, lo, hi, dmi);
}

// Host-memory verification of equations [lo, hi) on device di.  Batch mode (cert_offsets, the m + 1
// vote offsets of the call's certificates; msgs = their m digests): equation v checks digest c with
// offsets[c] <= v < offsets[c + 1], the index built on the device for large ranges.
int verify_range(int di, const uint8_t* msgs, uint64_t msg_stride, const uint32_t* cert_offsets,
                 const uint8_t* pks, const uint8_t* sigs, uint64_t lo, uint64_t hi, int strict,
                 std::vector<uint64_t>& out_words, uint64_t nmsgs) {
  DevCtx& d = *ctx(di);
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.hip_id));
  const uint64_t n = hi - lo;
  const uint64_t words = (n + 63) / 64;
  out_words.assign(words, 0);
  if (n == 0) return 0;
  const bool batch = cert_offsets != nullptr;
  uint64_t c_lo = 0, c_end = 0;
  if (batch) cert_span(cert_offsets, nmsgs, lo, hi, c_lo, c_end);
  const uint64_t msg_bytes = batch ? 32 * nmsgs : (msg_stride ? 32 * n : 32);
  const size_t need = align256(msg_bytes) + align256(batch ? 4 * n : 0) + align256(32 * n) + align256(64 * n) +
                      align256(8 * (words + 1));
  const size_t offs_bytes = batch ? 4 * (c_end - c_lo + 1) : 0;
  if (int rc = d.ensure_arena(need + align256(offs_bytes))) return rc;
  Carve c(d.arena);
  uint8_t* dm = c.take<uint8_t>(msg_bytes);
  uint32_t* dmi = batch ? c.take<uint32_t>(4 * n) : nullptr;
  uint8_t* dp = c.take<uint8_t>(32 * n);
  uint8_t* ds = c.take<uint8_t>(64 * n);
  uint64_t* dout = c.take<uint64_t>(8 * (words + 1));   // + the latency kernel's missing-key word
  uint32_t* doffs = batch ? c.take<uint32_t>(offs_bytes) : nullptr;   // large ranges: k_cert_index's input
  if (need <= NWC_PINNED_STAGE_MAX) {
    // small call (a certificate, a header): pack into pinned memory, one H2D, one D2H
    if (int rc = d.ensure_pinned(NWC_PINNED_STAGE_MAX)) return rc;
    uint8_t* h = d.pinned;
    std::memcpy(h + (dm - d.arena), batch ? msgs : msgs + (msg_stride ? 32 * lo : 0), msg_bytes);
    if (batch) fill_cert_index(reinterpret_cast<uint32_t*>(h + ((uint8_t*)dmi - d.arena)), cert_offsets, c_lo, c_end, lo, hi);
    std::memcpy(h + (dp - d.arena), pks + 32 * lo, 32 * n);
    std::memcpy(h + (ds - d.arena), sigs + 64 * lo, 64 * n);
    std::memset(h + ((uint8_t*)dout - d.arena), 0, 8 * (words + 1));
    int fl = LV_OUT_ZEROED;
    if (d.cm_n && g_hcm.all_cached(pks + 32 * lo, n)) fl |= LV_ALL_CACHED;
    else if (d.ak_n && n <= NWC_WIDE_MAX && d.ak_host.all_found(pks + 32 * lo, n)) fl |= LV_ALL_CACHED | LV_AUTO;
    const size_t vb_off = align256(need);   // byte verdicts of a zero-copy launch, after the staged inputs
    static const bool zero_copy = [] {
      const char* e = std::getenv("NWC_ZERO_COPY");
      return !(e && std::strcmp(e, "0") == 0);
    }();
    const bool zc_ok = zero_copy && n <= NWC_WIDE_MAX && vb_off + n <= NWC_PINNED_STAGE_MAX &&
                       verify_path() == VPath::Default;
    const bool zc_cached = zc_ok && (fl & LV_ALL_CACHED) && (fl & LV_AUTO ? d.ak_comb != nullptr : d.cm_comb != nullptr);
    const bool zc_cold = zc_ok && !(fl & LV_ALL_CACHED) && !d.cm_n && cold_path();
    if (zc_cached || zc_cold) {
      // every key cached: the latency kernel reads the staged inputs in place from pinned host
      // memory and stores one verdict byte per equation there -- no DMA copy either way; no key
      // cached (first sight): the cold kernel, the same way
      uint8_t* hb = h + vb_off;
      std::memset(hb, 0, n);
      auto dev = [&](const void* p) { return p ? d.pinned_dev + ((const uint8_t*)p - d.arena) : nullptr; };
      if (int rc = launch_verify(d, dev(dm), reinterpret_cast<const uint32_t*>(dev(dmi)), msg_stride ? 1 : 0, dev(dp),
                                 dev(ds), n, strict, dout, d.stream, fl, d.pinned_dev + (hb - h)))
        return rc;
      static const bool spin = [] {
        const char* e = std::getenv("NWC_SPIN_WAIT");   // 0 = wait for the stream (A/B)
        return !(e && std::strcmp(e, "0") == 0);
      }();
      if (spin) {
        // poll the verdict bytes (bit 7 = written); a launch that never writes them (a device
        // error) falls back to the stream wait after 200 ms, which reports the error
        const volatile uint8_t* vb = hb;
        const auto t0 = std::chrono::steady_clock::now();
        uint64_t done = 0;
        for (;;) {
          while (done < n && (vb[done] & 0x80u)) ++done;
          if (done == n) break;
          if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
            HIP_TRY(hipStreamSynchronize(d.stream));
            for (done = 0; done < n && (vb[done] & 0x80u); ++done) {}
            if (done != n) return set_err(NWC_ERR_DEVICE, "latency kernel left verdicts unwritten");
            break;
          }
          __builtin_ia32_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
      } else {
        HIP_TRY(hipStreamSynchronize(d.stream));
      }
      bool missing = false;
      for (uint64_t i = 0; i < n; ++i) {
        if (hb[i] & 1) out_words[i >> 6] |= 1ull << (i & 63);
        missing = missing || (hb[i] & 2);
      }
      if (!missing) return zc_cold ? auto_insert(d, pks + 32 * lo, n) : 0;
      // a key was missing on the device after all (cold: a reduction failed): stage the inputs
      // and run the general path
      std::fill(out_words.begin(), out_words.end(), 0);
      fl &= ~(LV_ALL_CACHED | LV_AUTO);
      HIP_TRY(hipMemcpyAsync(d.arena, h, (size_t)((uint8_t*)dout - d.arena) + 8 * (words + 1), hipMemcpyHostToDevice,
                             d.stream));
    } else {
      HIP_TRY(hipMemcpyAsync(d.arena, h, (size_t)((uint8_t*)dout - d.arena) + 8 * (words + 1), hipMemcpyHostToDevice,
                             d.stream));
    }
    if (int rc = launch_verify(d, dm, dmi, msg_stride ? 1 : 0, dp, ds, n, strict, dout, d.stream, fl)) return rc;
    HIP_TRY(hipMemcpyAsync(h, dout, 8 * (words + 1), hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    if ((fl & LV_ALL_CACHED) && h[8 * words] != 0) {
      // a key was missing on the device after all: the general path decides every equation
      if (int rc = launch_verify(d, dm, dmi, msg_stride ? 1 : 0, dp, ds, n, strict, dout, d.stream)) return rc;
      HIP_TRY(hipMemcpyAsync(h, dout, 8 * words, hipMemcpyDeviceToHost, d.stream));
      HIP_TRY(hipStreamSynchronize(d.stream));
    }
    std::memcpy(out_words.data(), h, 8 * words);
    if (!(fl & LV_ALL_CACHED) && n <= NWC_WIDE_MAX && verify_path() == VPath::Default)
      if (int rc = auto_insert(d, pks + 32 * lo, n)) return rc;
    return 0;
  }
  // Strict calls without a committee cache: the paired pipeline.  Chunks alternate between the
  // device stream and the side stream, each launch on its own half of the table slots with its own
  // fallback count and list region (PairLaunch), so chunk k + 1's blocks take the slots chunk k's
  // drain frees instead of waiting for its last block, and the first chunk can be small
  // (NWC_HOST_PAIR_FIRST, 65,536 equations = 8 MB of inputs, then x NWC_HOST_PAIR_GROWTH = 2).
  // The fallback passes run once the streams have joined.  NWC_HOST_PAIR=0: the single-stream
  // chunks below (A/B).
  static const bool pair_on = [] {
    const char* e = std::getenv("NWC_HOST_PAIR");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  static const uint64_t pair_first = [] {
    const char* e = std::getenv("NWC_HOST_PAIR_FIRST");
    return std::max<uint64_t>(64, (e ? std::strtoull(e, nullptr, 10) : 65536ull) / 64 * 64);
  }();
  static const uint64_t pair_growth = [] {
    const char* e = std::getenv("NWC_HOST_PAIR_GROWTH");
    return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : 2ull;
  }();
  static const uint64_t pair_max = [] {
    const char* e = std::getenv("NWC_HOST_PAIR_MAX");
    return std::max<uint64_t>(64, (e ? std::strtoull(e, nullptr, 10) : 1ull << 20) / 64 * 64);
  }();
  if (pair_on && strict && !batch && verify_path() == VPath::Default && !d.cm_n && n >= 2 * pair_first &&
      n <= verify_max_launch()) {
    if (int rc = ensure_stager(d)) return rc;
    if (int rc = ensure_verify_tables(d)) return rc;
    if (int rc = release_idle_buffers(d, d.pair_buf)) return rc;
    HostStager* const hs = d.stager.get();
    hs->reset();
    const auto tv0 = std::chrono::steady_clock::now();
    std::vector<uint64_t> cuts{0};
    uint64_t maxlen = 0;
    for (uint64_t len = pair_first; cuts.back() < n; len = std::min(len * pair_growth, std::max(pair_first, pair_max))) {
      uint64_t next = std::min<uint64_t>(n, cuts.back() + len);
      if (n - next < pair_first / 2) next = n;   // no sliver of a last chunk
      maxlen = std::max(maxlen, next - cuts.back());
      cuts.push_back(next);
    }
    const uint64_t nch = cuts.size() - 1;
    while (d.ev_chunk.size() < nch) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      d.ev_chunk.push_back(e);
    }
    // slots, lists and the per-chunk counts and list regions sized once, before any launch: inside
    // the pipeline nothing is reallocated under a running chunk (hold_lists: no shrink either)
    const uint64_t gcap = (uint64_t)d.cus * d.verify_blocks_per_cu * NWC_VERIFY_GRID_MULT;
    if (int rc = ensure_scratch(d, (size_t)gcap * 256 * 2 * nwc::TAB_BYTES_PER_LANE, maxlen)) return rc;
    const size_t counts_bytes = align256(4 * nch), pair_need = counts_bytes + 4 * n;
    if (pair_need > d.pair_cap) {
      HIP_TRY(hipEventSynchronize(d.scratch_free));
      if (d.pair_buf) HIP_TRY(hipFree(d.pair_buf));
      d.pair_buf = nullptr;
      d.pair_cap = 0;
      HIP_TRY(hipMalloc(&d.pair_buf, pair_need));
      d.pair_cap = pair_need;
    }
    uint32_t* const counts = reinterpret_cast<uint32_t*>(d.pair_buf);
    uint32_t* const lists = reinterpret_cast<uint32_t*>(d.pair_buf + counts_bytes);
    struct Hold {
      DevCtx& d;
      ~Hold() {
        d.hold_lists = false;
        d.busy_buf = nullptr;
      }
    } hold{d};
    d.hold_lists = true;
    d.busy_buf = d.pair_buf;
    // the previous call's kernels may still read the arena and the slots: the copies wait for the
    // device stream, both compute streams for scratch_free
    HIP_TRY(hipEventRecord(d.ev_fork, d.stream));
    HIP_TRY(hipStreamWaitEvent(d.xfer, d.ev_fork, 0));
    HIP_TRY(hipStreamWaitEvent(d.side, d.ev_fork, 0));
    HIP_TRY(hipStreamWaitEvent(d.stream, d.scratch_free, 0));
    HIP_TRY(hipStreamWaitEvent(d.side, d.scratch_free, 0));
    auto h2d = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
      return hs->put(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), bytes);
    };
    if (!msg_stride) HIP_TRY(h2d(dm, msgs, 32));
    for (uint64_t k = 0; k < nch; ++k) {
      const uint64_t c0 = cuts[k], len = cuts[k + 1] - cuts[k];
      if (msg_stride) HIP_TRY(h2d(dm + 32 * c0, msgs + 32 * (lo + c0), 32 * len));
      HIP_TRY(h2d(dp + 32 * c0, pks + 32 * (lo + c0), 32 * len));
      HIP_TRY(h2d(ds + 64 * c0, sigs + 64 * (lo + c0), 64 * len));
      HIP_TRY(hs->flush());
      HIP_TRY(hipEventRecord(d.ev_chunk[k], d.xfer));
      const hipStream_t sk = (k & 1) ? d.side : d.stream;
      HIP_TRY(hipStreamWaitEvent(sk, d.ev_chunk[k], 0));
      const PairLaunch pl{(int)(k & 1), lists + c0, counts + k};
      if (int rc = launch_verify(d, msg_stride ? dm + 32 * c0 : dm, nullptr, msg_stride ? 1 : 0, dp + 32 * c0,
                                 ds + 64 * c0, len, strict, dout + c0 / 64, sk, 0, nullptr, 0, &pl))
        return rc;
    }
    HIP_TRY(hipEventRecord(d.ev_join, d.side));
    HIP_TRY(hipStreamWaitEvent(d.stream, d.ev_join, 0));
    // every chunk's failed reductions (rare: waves exit at once on an empty list)
    for (uint64_t k = 0; k < nch; ++k) {
      const uint64_t c0 = cuts[k], len = cuts[k + 1] - cuts[k];
      const nwc::VerifyArgs a{msg_stride ? dm + 32 * c0 : dm, nullptr, msg_stride ? 1u : 0u, dp + 32 * c0, ds + 64 * c0,
                              dout + c0 / 64, len, strict, d.base_table, d.base24, d.scratch, lists + c0, counts + k,
                              0u, nwc::Committee{}};
      hipLaunchKernelGGL(nwc::k_verify_fallback, dim3(16), dim3(256), 0, d.stream, a);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(d.scratch_free, d.stream));
    const auto tq = std::chrono::steady_clock::now();
    HIP_TRY(hipMemcpyAsync(out_words.data(), dout, 8 * words, hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    if (host_timing())
      std::fprintf(stderr, "nwc host call (paired): %llu equations in %llu chunks: copies queued after %.2f ms, done %.2f ms later\n",
                   (unsigned long long)n, (unsigned long long)nch, std::chrono::duration<double>(tq - tv0).count() * 1e3,
                   std::chrono::duration<double>(std::chrono::steady_clock::now() - tq).count() * 1e3);
    return 0;
  }
  static const uint64_t chunk = [] {
    const char* e = std::getenv("NWC_HOST_CHUNK");   // 0 = no pipelining (A/B)
    return e ? (uint64_t)std::strtoull(e, nullptr, 10) / 64 * 64 : (uint64_t)NWC_HOST_CHUNK;
  }();
  static const uint64_t growth = [] {
    const char* e = std::getenv("NWC_HOST_CHUNK_GROWTH");   // 1 = equal chunks (A/B)
    return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : (uint64_t)NWC_HOST_CHUNK_GROWTH;
  }();
  if (chunk && n >= 2 * chunk) {
    // pipelined: inputs of chunk k on the transfer stream, its verification on the device stream
    // after the chunk's event; every chunk has its own region of the arena (no reuse hazards).
    // Chunk k + 1 is up to `growth` x chunk k: its 128 B per equation cross PCIe (~50 GB/s) while
    // chunk k verifies (~100 M/s), so it arrives in time while growing up to ~3.7x; fewer, larger
    // launches leave fewer kernel tails (the first chunk is one round of resident lanes).
    if (int rc = ensure_stager(d)) return rc;
    // copies of one chunk's inputs: through the pinned stages
    HostStager* const hs = d.stager.get();
    hs->reset();
    const auto tv0 = std::chrono::steady_clock::now();
    auto h2d = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
      return hs->put(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), bytes);
    };
    std::vector<uint64_t> cuts{0};
    // chunks stop growing at NWC_HOST_CHUNK_MAX equations: when the kernels keep pace with the
    // copies (the comb kernel: ~640 M votes/s against ~600 M votes/s of inputs through the stages)
    // a huge last chunk would start only once all its inputs are in and run alone at the end
    static const uint64_t chunk_max = [] {
      const char* e = std::getenv("NWC_HOST_CHUNK_MAX");   // A/B
      return e ? std::max<uint64_t>(64, std::strtoull(e, nullptr, 10)) : (uint64_t)NWC_HOST_CHUNK_MAX;
    }();
    for (uint64_t len = chunk; cuts.back() < n; len = std::min(len * growth, std::max(chunk, chunk_max))) {
      uint64_t next = std::min<uint64_t>(n, cuts.back() + len);
      if (n - next < chunk / 2) next = n;   // no sliver of a last chunk
      cuts.push_back(next);
    }
    const uint64_t nch = cuts.size() - 1;
    while (d.ev_chunk.size() < nch) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      d.ev_chunk.push_back(e);
    }
    // Chunks on the comb path (launch keys or the committee cache) defer their sign tests: a
    // lane gets ~8 votes of a 1M-vote chunk, and its one inversion would be ~9 % of each vote's
    // work (k_verify_comb_y; the sign pass of chunk k runs in the first blocks of chunk k + 1's
    // launch, the last one alone; SignRecs of two chunks alternate in sign_buf)
    uint64_t maxlen = 0;
    for (uint64_t k = 0; k < nch; ++k) maxlen = std::max(maxlen, cuts[k + 1] - cuts[k]);
    const bool ysplit = !strict && sign_defer();
    nwc::SignRecs reg[2] = {};
    if (ysplit) {
      if (int rc = release_idle_buffers(d, d.sign_buf)) return rc;
      const size_t per = align256(32 * maxlen);
      const size_t need_s = 2 * (3 * per + align256(4 * maxlen));
      if (need_s > d.sign_cap) {
        HIP_TRY(hipEventSynchronize(d.scratch_free));
        if (d.sign_buf) HIP_TRY(hipFree(d.sign_buf));
        d.sign_buf = nullptr;
        d.sign_cap = 0;
        HIP_TRY(hipMalloc(&d.sign_buf, need_s));
        d.sign_cap = need_s;
      }
      Carve cs(d.sign_buf);
      for (auto& r : reg) {
        r.x = cs.take<uint32_t>(32 * maxlen);
        r.z = cs.take<uint32_t>(32 * maxlen);
        r.p = cs.take<uint32_t>(32 * maxlen);
        r.meta = cs.take<uint32_t>(4 * maxlen);
      }
    }
    uint64_t owed_c0 = 0, owed_len = 0;   // the chunk whose sign tests are still to run
    int owed_reg = 0;
    struct Busy {
      DevCtx& d;
      ~Busy() { d.busy_buf = nullptr; }
    } busy{d};
    d.busy_buf = d.sign_buf;
    // the previous call's kernels may still read the arena: the transfers wait for the stream
    HIP_TRY(hipEventRecord(d.ev_fork, d.stream));
    HIP_TRY(hipStreamWaitEvent(d.xfer, d.ev_fork, 0));
    if (batch) {
      // digests and offsets first; the vote index is built on the device behind them, so chunk 0's
      // event (recorded later on the same stream) covers it
      HIP_TRY(h2d(dm, msgs, msg_bytes));
      HIP_TRY(h2d(doffs, cert_offsets + c_lo, offs_bytes));
      HIP_TRY(hs->flush());
      launch_cert_index(doffs, c_lo, c_end, lo, hi, dmi, d.xfer);
      HIP_TRY(hipGetLastError());
    } else if (!msg_stride) {
      HIP_TRY(h2d(dm, msgs, 32));
    }
    for (uint64_t k = 0; k < nch; ++k) {
      const uint64_t c0 = cuts[k], len = cuts[k + 1] - cuts[k];
      if (msg_stride) HIP_TRY(h2d(dm + 32 * c0, msgs + 32 * (lo + c0), 32 * len));
      HIP_TRY(h2d(dp + 32 * c0, pks + 32 * (lo + c0), 32 * len));
      HIP_TRY(h2d(ds + 64 * c0, sigs + 64 * (lo + c0), 64 * len));
      HIP_TRY(hs->flush());
      HIP_TRY(hipEventRecord(d.ev_chunk[k], d.xfer));
      HIP_TRY(hipStreamWaitEvent(d.stream, d.ev_chunk[k], 0));
      const nwc::SignPass sp{sign_recs_at(reg[owed_reg], -(int64_t)owed_c0), owed_c0, owed_len, dout,
                             comb_sign_blocks(d, owed_len)};
      const bool y = ysplit && takes_comb_path(d, len, strict);
      if (!y && owed_len) {
        if (int rc = launch_comb_sign(d, sp.rec, owed_c0, owed_len, dout, d.stream)) return rc;
        owed_len = 0;
      }
      const int r = (int)(k & 1);
      if (int rc = launch_verify(d, msg_stride ? dm + 32 * c0 : dm, batch ? dmi + c0 : nullptr, msg_stride ? 1 : 0,
                                 dp + 32 * c0, ds + 64 * c0, len, strict, dout + c0 / 64, d.stream, 0, nullptr, 0,
                                 nullptr, y ? &reg[r] : nullptr, y && owed_len ? &sp : nullptr))
        return rc;
      if (y) {
        owed_c0 = c0;
        owed_len = len;
        owed_reg = r;
      }
    }
    if (owed_len)
      if (int rc = launch_comb_sign(d, sign_recs_at(reg[owed_reg], -(int64_t)owed_c0), owed_c0, owed_len, dout, d.stream))
        return rc;
    const auto tq = std::chrono::steady_clock::now();
    HIP_TRY(hipMemcpyAsync(out_words.data(), dout, 8 * words, hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    if (host_timing())
      std::fprintf(stderr, "nwc host call: %llu equations in %llu chunks: copies queued after %.2f ms, done %.2f ms later\n",
                   (unsigned long long)n, (unsigned long long)nch, std::chrono::duration<double>(tq - tv0).count() * 1e3,
                   std::chrono::duration<double>(std::chrono::steady_clock::now() - tq).count() * 1e3);
    return 0;
  }
  if (batch) {
    HIP_TRY(hipMemcpyAsync(dm, msgs, msg_bytes, hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(doffs, cert_offsets + c_lo, offs_bytes, hipMemcpyHostToDevice, d.stream));
    launch_cert_index(doffs, c_lo, c_end, lo, hi, dmi, d.stream);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemcpyAsync(dm, msgs + (msg_stride ? 32 * lo : 0), msg_bytes, hipMemcpyHostToDevice, d.stream));
  }
  HIP_TRY(hipMemcpyAsync(dp, pks + 32 * lo, 32 * n, hipMemcpyHostToDevice, d.stream));
  HIP_TRY(hipMemcpyAsync(ds, sigs + 64 * lo, 64 * n, hipMemcpyHostToDevice, d.stream));
  if (int rc = launch_verify(d, dm, dmi, msg_stride ? 1 : 0, dp, ds, n, strict, dout, d.stream)) return rc;
  HIP_TRY(hipMemcpyAsync(out_words.data(), dout, 8 * words, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  return 0;
}

// A per-launch device buffer of the batch entries (MSM, Straus, resolve), grown on demand and
// shrunk back when it holds more than NWC_VERIFY_KEEP_BYTES and a launch needs under a quarter of
// it (a primary and workers share the GPU: worker/src/worker.rs:182,227).  Every launch that uses
// these buffers records scratch_free after its last kernel, so waiting for it (and for s) drains
// their users on any stream before the buffer is replaced.
int ensure_buf(DevCtx& d, uint8_t*& p, size_t& cap, size_t need, hipStream_t s) {
  const bool shrink = cap > verify_keep_bytes() && need < cap / 4;
  if (need <= cap && !shrink) return 0;
  HIP_TRY(hipEventSynchronize(d.scratch_free));
  HIP_TRY(hipStreamSynchronize(s));
  if (p) HIP_TRY(hipFree(p));
  p = nullptr;
  cap = 0;
  HIP_TRY(hipMalloc(&p, need));
  cap = need;
  return 0;
}

// The per-launch z_i seed: 32 bytes from the host's CSPRNG (dalek: merlin transcript + thread_rng),
// or the test knob's fixed value (nwc_diag_set("dalek_seed")).
void draw_seed(uint32_t seed[8]) {
  const uint64_t fixed = knobs().dalek_seed.load();
  if (fixed) {
    for (int i = 0; i < 8; ++i) seed[i] = i == 0 ? (uint32_t)fixed : 0u;
    return;
  }
  static thread_local std::random_device rd;
  for (int i = 0; i < 8; ++i) seed[i] = rd();
}

int ensure_straus_scratch(DevCtx& d, size_t bytes, hipStream_t s) {
  if (int rc = release_idle_buffers(d, d.straus_scratch)) return rc;
  return ensure_buf(d, d.straus_scratch, d.straus_cap, bytes, s);
}

// dalek's batch equation over sub-batches (k_verify_straus) + the exact leaves for the failing
// sub-batches, on d's stream s: leaf words (a bit per vote) for cert_reduce.  Caller holds d.mu
// and has set the device.
int launch_straus(DevCtx& d, const uint8_t* dig, const uint32_t* mi, const uint8_t* pks, const uint8_t* sigs,
                  uint64_t nvotes, uint64_t* leaf, hipStream_t s) {
  if (nvotes == 0) return 0;
  if (int rc = ensure_verify_tables(d)) return rc;
  if (nvotes > verify_max_launch()) {
    // consecutive launches of at most NWC_VERIFY_MAX_LAUNCH votes, as launch_verify: sub-batches
    // are any consecutive votes (each reads its own certificate's digest through mi)
    const uint64_t step = verify_max_launch();
    for (uint64_t lo = 0; lo < nvotes; lo += step)
      if (int rc = launch_straus(d, dig, mi + lo, pks + 32 * lo, sigs + 64 * lo, std::min(step, nvotes - lo), leaf + lo / 64, s))
        return rc;
    return 0;
  }
  if (!d.comb16)   // no basepoint comb (NWC_COMB16=0): the exact leaves
    return launch_verify(d, dig, mi, 0, pks, sigs, nvotes, 0, leaf, s);
  // sub-batches of ~12 votes (knobs().straus_nq), every lane slot the same number of rounds
  const uint32_t target = knobs().straus_nq.load();
  const uint64_t resident = (uint64_t)d.cus * nwc::STRAUS_WAVES_PER_SIMD * 256;
  const uint64_t runs = nwc::straus_runs(nvotes, resident, target);
  const uint64_t lanes = std::min<uint64_t>((runs + 255) / 256 * 256, resident);
  const uint64_t maxq = (nvotes + runs - 1) / runs;
  const uint64_t stride = maxq * nwc::STRAUS_VOTE_BYTES;
  if (int rc = ensure_straus_scratch(d, lanes * stride, s)) return rc;
  // the failing sub-batches' leaves: the list-mode leaf kernel's scratch and lists
  const uint64_t lgrid = (uint64_t)d.cus * d.verify_blocks_per_cu;
  if (int rc = ensure_scratch(d, (size_t)lgrid * 256 * 2 * nwc::TAB_BYTES_PER_LANE, nvotes)) return rc;
  HIP_TRY(hipStreamWaitEvent(s, d.scratch_free, 0));
  nwc::StrausArgs sa{};
  sa.digests = dig; sa.msg_index = mi; sa.pks = pks; sa.sigs = sigs; sa.nv = nvotes; sa.runs = runs;
  draw_seed(sa.seed);
  sa.comb16 = d.comb16; sa.scratch = d.straus_scratch; sa.lane_stride = stride;
  sa.leaf_words = leaf; sa.list = d.uc_list; sa.count = d.uc_count;
  HIP_TRY(hipMemsetAsync(leaf, 0, 8 * ((nvotes + 63) / 64), s));
  HIP_TRY(hipMemsetAsync(d.uc_count, 0, sizeof(uint32_t), s));
  HIP_TRY(hipMemsetAsync(d.fb_count, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(nwc::k_verify_straus<false>, dim3((unsigned)(lanes / 256)), dim3(256), 0, s, sa);
  HIP_TRY(hipGetLastError());
  nwc::VerifyArgs a{dig, mi, 0, pks, sigs, leaf, nvotes, 0, d.base_table, d.base24, d.scratch, d.fb_list,
                    d.fb_count, 0u, nwc::Committee{}};
  const nwc::CombArgs ca{d.uc_list, d.uc_count, d.comb_base, d.comb16};
  hipLaunchKernelGGL((nwc::k_verify<true, false, true>), dim3((unsigned)lgrid), dim3(256), 0, s, a, ca);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(nwc::k_verify_fallback, dim3(16), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  if (int rc = launch_torsion(d, pks, leaf, nvotes, d.uc_list, d.uc_count, nwc::Committee{}, s)) return rc;
  HIP_TRY(hipEventRecord(d.scratch_free, s));
  return 0;
}


// dalek's batch equation over groups of consecutive votes as a Pippenger MSM with a wavefront-level
// bucket reduction (k_verify_msm, msm.h) + the exact leaves for the groups it rejects, on d's
// stream s: leaf words (a bit per vote) for cert_reduce, like launch_straus.  Caller holds d.mu and
// has set the device.
int launch_msm(DevCtx& d, const uint8_t* dig, const uint32_t* mi, const uint8_t* pks, const uint8_t* sigs,
               uint64_t nvotes, uint64_t* leaf, hipStream_t s) {
  if (nvotes == 0) return 0;
  if (int rc = ensure_verify_tables(d)) return rc;
  if (nvotes > verify_max_launch()) {
    const uint64_t step = verify_max_launch();
    for (uint64_t lo = 0; lo < nvotes; lo += step)
      if (int rc = launch_msm(d, dig, mi + lo, pks + 32 * lo, sigs + 64 * lo, std::min(step, nvotes - lo), leaf + lo / 64, s))
        return rc;
    return 0;
  }
  if (!d.comb16)   // no basepoint comb (NWC_COMB16=0): the exact leaves
    return launch_verify(d, dig, mi, 0, pks, sigs, nvotes, 0, leaf, s);
  static int bpc = [] {
    int b = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(nwc::k_verify_msm), 64, 0);
    return b > 0 ? b : 1;
  }();
  const uint64_t slots = (uint64_t)d.cus * bpc;   // resident waves (one group each at a time)
  uint32_t group = knobs().msm_group.load();
  if (group == 0) {
    // as few rounds of the resident waves as groups of <= MSM_GMAX allow, every round full: the
    // per-window costs of a group (scan, doublings, key points) amortise over larger groups, and a
    // partial last round would leave waves idle
    const uint64_t rounds = (nvotes + slots * nwc::MSM_GMAX - 1) / (slots * nwc::MSM_GMAX);
    group = (uint32_t)((nvotes + slots * rounds - 1) / (slots * rounds));
  }
  group = std::min<uint32_t>(nwc::MSM_GMAX, std::max<uint32_t>(64, (group + 63) / 64 * 64));
  const uint64_t groups = (nvotes + group - 1) / group;
  const uint64_t grid = std::min<uint64_t>(groups, slots);
  // per-wave points and digits, then the failing groups' vote list (count word, entries)
  const size_t list_off = align256((size_t)grid * nwc::MSM_WAVE_BYTES);
  const size_t need = list_off + 256 + 4 * nvotes;
  if (int rc = release_idle_buffers(d, d.msm_scratch)) return rc;
  if (int rc = ensure_buf(d, d.msm_scratch, d.msm_cap, need, s)) return rc;
  if (!d.msm_stats) {
    HIP_TRY(hipMalloc(&d.msm_stats, 4 * nwc::MSM_ST_WORDS));
    HIP_TRY(hipMemsetAsync(d.msm_stats, 0, 4 * nwc::MSM_ST_WORDS, s));
  }
  uint32_t* const mcount = reinterpret_cast<uint32_t*>(d.msm_scratch + list_off);
  uint32_t* const mlist = mcount + 64;
  // the failing groups' votes go straight to the exact leaves (list mode): a vote meets at most one
  // random equation, its group's
  const uint64_t lgrid = (uint64_t)d.cus * d.verify_blocks_per_cu;
  if (int rc = ensure_scratch(d, (size_t)lgrid * 256 * 2 * nwc::TAB_BYTES_PER_LANE, nvotes)) return rc;
  HIP_TRY(hipStreamWaitEvent(s, d.scratch_free, 0));
  nwc::MsmArgs ma{};
  ma.digests = dig; ma.msg_index = mi; ma.pks = pks; ma.sigs = sigs; ma.nv = nvotes; ma.group = group;
  draw_seed(ma.seed);
  ma.comb16 = d.comb16; ma.scratch = d.msm_scratch;
  ma.leaf_words = leaf; ma.list = mlist; ma.count = mcount; ma.stats = d.msm_stats;
  HIP_TRY(hipMemsetAsync(leaf, 0, 8 * ((nvotes + 63) / 64), s));
  HIP_TRY(hipMemsetAsync(mcount, 0, sizeof(uint32_t), s));
  HIP_TRY(hipMemsetAsync(d.fb_count, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(nwc::k_verify_msm, dim3((unsigned)grid), dim3(64), 0, s, ma);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(nwc::k_msm_policy, dim3(1), dim3(64), 0, s, d.msm_stats, (uint32_t)knobs().msm_adapt.load());
  HIP_TRY(hipGetLastError());
  const nwc::VerifyArgs a{dig, mi, 0, pks, sigs, leaf, nvotes, 0, d.base_table, d.base24, d.scratch, d.fb_list,
                          d.fb_count, 0u, nwc::Committee{}};
  const nwc::CombArgs ca{mlist, mcount, d.comb_base, d.comb16};
  hipLaunchKernelGGL((nwc::k_verify<true, false, true>), dim3((unsigned)lgrid), dim3(256), 0, s, a, ca);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(nwc::k_verify_fallback, dim3(16), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  if (int rc = launch_torsion(d, pks, leaf, nvotes, mlist, mcount, nwc::Committee{}, s)) return rc;
  HIP_TRY(hipEventRecord(d.scratch_free, s));
  return 0;
}

// dalek's batch equation per certificate over the votes the leaves rejected (resolve.h), on s after
// the leaves wrote `leaf` (bit per vote of m certificates): cm = the key set whose combs the leaves
// used (nullptr combs: the ladder).  Sets the bits of the failing votes of certificates the equation
// accepts.  Caller holds d.mu and has set the device.
int launch_resolve(DevCtx& d, const uint8_t* dig, const uint32_t* mi, uint64_t m, const uint8_t* pks,
                   const uint8_t* sigs, uint64_t nv, uint64_t* leaf, const nwc::Committee& cm, hipStream_t s) {
  if (nv == 0) return 0;
  if (nv > 0xFFFFFFFFull || m > 0xFFFFFFFFull) return set_err(NWC_ERR_ARG, "more than 2^32 - 1 votes or certificates");
  const size_t state_off = align256(256 + 4 * (size_t)nv);
  if (int rc = release_idle_buffers(d, d.rs_buf)) return rc;
  if (int rc = ensure_buf(d, d.rs_buf, d.rs_cap, state_off + align256(4 * (size_t)m), s)) return rc;
  // one lane per failing vote; a lane slot's ladder table lives in the verification scratch
  const uint64_t grid = (uint64_t)d.cus * d.verify_blocks_per_cu;
  if (int rc = ensure_scratch(d, (size_t)grid * 256 * 2 * nwc::TAB_BYTES_PER_LANE, std::min(nv, verify_max_launch())))
    return rc;
  HIP_TRY(hipStreamWaitEvent(s, d.scratch_free, 0));
  uint32_t* const count = reinterpret_cast<uint32_t*>(d.rs_buf);
  uint32_t* const list = count + 64;
  uint32_t* const state = reinterpret_cast<uint32_t*>(d.rs_buf + state_off);
  HIP_TRY(hipMemsetAsync(count, 0, sizeof(uint32_t), s));
  HIP_TRY(hipMemsetAsync(state, 0, 4 * (size_t)m, s));
  const uint64_t words = (nv + 63) / 64;
  hipLaunchKernelGGL(nwc::k_list_failing, dim3((unsigned)std::min<uint64_t>((words + 255) / 256, (uint64_t)d.cus * 8)),
                     dim3(256), 0, s, leaf, nv, list, count);
  HIP_TRY(hipGetLastError());
  nwc::ResolveArgs ra{};
  ra.digests = dig; ra.msg_index = mi; ra.pks = pks; ra.sigs = sigs; ra.list = list; ra.count = count;
  draw_seed(ra.seed);
  ra.cm = cm; ra.comb16 = d.comb16; ra.base_table = d.base_table; ra.scratch = d.scratch;
  ra.cert_state = state; ra.leaf_words = leaf;
  hipLaunchKernelGGL(nwc::k_vote_resolve, dim3((unsigned)grid), dim3(256), 0, s, ra);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(nwc::k_resolve_apply, dim3((unsigned)(d.cus * 2)), dim3(256), 0, s, ra);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(d.scratch_free, s));
  return 0;
}

// Signature::verify_batch over m certificates with dalek's batch semantics (crypto/src/lib.rs:218).
// Where key combs apply (a committee cache with combs, or a launch large enough for launch keys):
// the exact per-vote leaves on the comb path, then dalek's equation once per certificate over the
// votes they rejected (launch_resolve) -- every vote meets one random equation, its certificate's.
// Otherwise the Pippenger groups first (launch_msm).  Caller holds d.mu and has set the device.
int launch_batch_dalek(DevCtx& d, const uint8_t* dig, const uint32_t* mi, uint64_t m, const uint8_t* pks,
                       const uint8_t* sigs, uint64_t nv, uint64_t* leaf, hipStream_t s) {
  if (nv == 0) return 0;
  if (int rc = ensure_verify_tables(d)) return rc;
  const bool committee = d.cm_n && d.cm_comb;
  const bool lkeys = !d.cm_n && nv >= nwc::LK_MIN_EQUATIONS && knobs().launch_keys.load();
  if (verify_path() != VPath::Default || !d.comb16 || !(committee || lkeys))
    return launch_msm(d, dig, mi, pks, sigs, nv, leaf, s);
  if (int rc = launch_verify(d, dig, mi, 0, pks, sigs, nv, 0, leaf, s)) return rc;
  const nwc::Committee cm = committee ? nwc::Committee{d.cm_keys, d.cm_flags, d.cm_tables, d.cm_comb, d.cm_slots,
                                                       d.cm_slot_mask, d.cm_n}
                                      : nwc::Committee{d.lk.keys, d.lk.flags, nullptr, d.lk.comb, d.lk.slots,
                                                       nwc::LK_SLOTS - 1, nwc::LK_MAX_KEYS};
  return launch_resolve(d, dig, mi, m, pks, sigs, nv, leaf, cm, s);
}

// Per-vote leaf bits of every device's share (whole certificates) -> certificate verdicts and the
// bad-vote bitmap (a certificate passes iff every vote's bit is set; an empty one passes).
int batch_verdicts(const uint32_t* offsets, size_t m, const std::vector<uint64_t>& cuts,
                   const std::vector<std::vector<uint64_t>>& parts, uint8_t* cert_ok_bitmap, uint8_t* bad_vote_bitmap) {
  // word-level: a certificate is ok iff every bit of its vote range is set (two masked words for a
  // 67-vote certificate), and the bad-vote bitmap is the complement of the leaf bits
  const uint64_t nv = offsets[m];
  std::vector<uint64_t> leafw((nv + 63) / 64 + 1, 0);
  uint8_t* const leafbytes = reinterpret_cast<uint8_t*>(leafw.data());
  for (size_t i = 0; i + 1 < cuts.size(); ++i) merge_bits(leafbytes, cuts[i], parts[i], cuts[i + 1] - cuts[i]);
  std::memset(cert_ok_bitmap, 0, (m + 7) / 8);
  for (size_t c = 0; c < m; ++c) {
    const uint64_t a = offsets[c], e = offsets[c + 1];
    bool ok = true;
    if (e > a) {
      const uint64_t w0 = a >> 6, w1 = (e - 1) >> 6;
      for (uint64_t w = w0; w <= w1 && ok; ++w) {
        uint64_t mask = ~0ull;
        if (w == w0) mask &= ~0ull << (a & 63);
        if (w == w1) mask &= ~0ull >> (63 - ((e - 1) & 63));
        ok = (leafw[w] & mask) == mask;
      }
    }
    if (ok) cert_ok_bitmap[c >> 3] |= (uint8_t)(1u << (c & 7));
  }
  if (bad_vote_bitmap && nv) {
    const uint64_t full = nv / 8;
    for (uint64_t i = 0; i < full; ++i) bad_vote_bitmap[i] = (uint8_t)~leafbytes[i];
    for (uint64_t v = full * 8; v < nv; ++v) {
      const bool bad = !((leafbytes[v >> 3] >> (v & 7)) & 1);
      bad_vote_bitmap[v >> 3] = (uint8_t)((bad_vote_bitmap[v >> 3] & ~(1u << (v & 7))) | ((unsigned)bad << (v & 7)));
    }
  }
  return 0;
}

// One device's share of nwc_verify_batch_straus_many: votes [lo, hi) (whole certificates) staged
// into the arena with one H2D each, the Straus launch, one D2H of the leaf words.
int straus_range(int di, const uint8_t* digests, size_t m, const uint32_t* offsets, const uint8_t* pks,
                 const uint8_t* sigs, uint64_t lo, uint64_t hi, std::vector<uint64_t>& out_words, bool msm = false) {
  DevCtx& d = *ctx(di);
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.hip_id));
  const uint64_t n = hi - lo;
  const uint64_t words = (n + 63) / 64;
  out_words.assign(words, 0);
  if (n == 0) return 0;
  uint64_t c_lo, c_end;
  cert_span(offsets, m, lo, hi, c_lo, c_end);
  const size_t offs_bytes = 4 * (c_end - c_lo + 1);
  const size_t need = align256(32 * m) + align256(4 * n) + align256(32 * n) + align256(64 * n) + align256(8 * words) +
                      align256(offs_bytes);
  if (int rc = d.ensure_arena(need)) return rc;
  Carve c(d.arena);
  uint8_t* dm = c.take<uint8_t>(32 * m);
  uint32_t* dmi = c.take<uint32_t>(4 * n);
  uint8_t* dp = c.take<uint8_t>(32 * n);
  uint8_t* ds = c.take<uint8_t>(64 * n);
  uint64_t* dout = c.take<uint64_t>(8 * words);
  uint32_t* doffs = c.take<uint32_t>(offs_bytes);
  HIP_TRY(hipMemcpyAsync(dm, digests, 32 * m, hipMemcpyHostToDevice, d.stream));
  HIP_TRY(hipMemcpyAsync(doffs, offsets + c_lo, offs_bytes, hipMemcpyHostToDevice, d.stream));
  launch_cert_index(doffs, c_lo, c_end, lo, hi, dmi, d.stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(dp, pks + 32 * lo, 32 * n, hipMemcpyHostToDevice, d.stream));
  HIP_TRY(hipMemcpyAsync(ds, sigs + 64 * lo, 64 * n, hipMemcpyHostToDevice, d.stream));
  if (int rc = msm ? launch_batch_dalek(d, dm, dmi, m, dp, ds, n, dout, d.stream)
                   : launch_straus(d, dm, dmi, dp, ds, n, dout, d.stream))
    return rc;
  HIP_TRY(hipMemcpyAsync(out_words.data(), dout, 8 * words, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  return 0;
}

}  // namespace

extern "C" {

int nwc_shard_bounds(uint64_t n, uint32_t world, uint32_t rank, uint64_t* lo, uint64_t* hi) {
  if (!lo || !hi || world == 0 || rank >= world) return set_err(NWC_ERR_ARG, "bad shard arguments");
  const uint64_t words = (n + 63) / 64, per = (words + world - 1) / world;
  *lo = std::min<uint64_t>(n, (uint64_t)rank * per * 64);
  *hi = std::min<uint64_t>(n, ((uint64_t)rank + 1) * per * 64);
  return 0;
}

int nwc_cert_cuts(const uint32_t* offsets, size_t m, uint32_t world, uint64_t* cuts) {
  if (!offsets || !cuts || world == 0) return set_err(NWC_ERR_ARG, "bad cut arguments");
  const uint64_t nv = offsets[m];
  cuts[0] = 0;
  size_t c = 0;
  for (uint32_t r = 1; r < world; ++r) {
    const uint64_t target = nv * r / world;
    while (c < m && offsets[c] < target) ++c;   // first boundary at or past the target
    cuts[r] = offsets[c];
  }
  cuts[world] = nv;
  return 0;
}

int nwc_version(void) { return (1 << 16) | 1; }

#ifndef NWC_BUILD_ID
#define NWC_BUILD_ID "unknown"
#endif
// "NWC_BUILD_ID:" + the hash narwhal_amd/build.py takes over the sources and flags; build.py finds
// it in the .so's bytes to decide whether the library is HEAD's.
static const char k_build_id[] = "NWC_BUILD_ID:" NWC_BUILD_ID;
const char* nwc_build_id(void) { return k_build_id + 13; }

int nwc_diag_set(const char* name, int64_t value) {
  if (!name) return set_err(NWC_ERR_ARG, "null knob name");
  if (value < 0 || value > 0xFFFFFFFFll) return set_err(NWC_ERR_ARG, "knob value out of range");
  if (std::strcmp(name, "straus_nq") == 0) {
    if (value < 1 || value > nwc::STRAUS_MAX_PER_LANE) return set_err(NWC_ERR_ARG, "straus_nq must be in [1, %d]", nwc::STRAUS_MAX_PER_LANE);
    knobs().straus_nq = (uint32_t)value;
  } else if (std::strcmp(name, "msm_group") == 0) {
    if (value != 0 && (value < 64 || value > nwc::MSM_GMAX || value % 64))
      return set_err(NWC_ERR_ARG, "msm_group must be 0 (sized per launch) or a multiple of 64 in [64, %d]", nwc::MSM_GMAX);
    knobs().msm_group = (uint32_t)value;
  } else if (std::strcmp(name, "msm_adapt") == 0) {
    if (value > 1) return set_err(NWC_ERR_ARG, "msm_adapt must be 0 or 1");
    knobs().msm_adapt = (uint32_t)value;
  } else if (std::strcmp(name, "dalek_seed") == 0) {
    knobs().dalek_seed = (uint64_t)value;
  } else if (std::strcmp(name, "launch_keys") == 0) {
    if (value > 1) return set_err(NWC_ERR_ARG, "launch_keys must be 0 or 1");
    knobs().launch_keys = (uint32_t)value;
  } else if (std::strcmp(name, "force_windows") == 0) {
    if (value != 0 && (value < nwc::HALF_WINDOWS_MIN || value > nwc::HALF_WINDOWS_MAX))
      return set_err(NWC_ERR_ARG, "force_windows must be 0 or in [%d, %d]", nwc::HALF_WINDOWS_MIN, nwc::HALF_WINDOWS_MAX);
    knobs().force_windows = (uint32_t)value;
  } else {
    return set_err(NWC_ERR_ARG, "unknown knob '%s'", name);
  }
  return 0;
}

const char* nwc_last_error(void) { return t_err.c_str(); }

int nwc_init(uint32_t device_mask) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_devs.empty()) return 0;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0)
    return set_err(NWC_ERR_NO_DEVICE, "no HIP device visible (%s)", hipGetErrorString(e));
  if (device_mask == 0) device_mask = 1;
  for (int i = 0; i < count && i < 32; ++i) {
    if (!((device_mask >> i) & 1)) continue;
    auto d = std::make_unique<DevCtx>();
    d->hip_id = i;
    if (int rc = init_device(*d)) { g_devs.clear(); return rc; }
    g_devs.push_back(std::move(d));
  }
  if (g_devs.empty()) return set_err(NWC_ERR_NO_DEVICE, "device mask 0x%x selects no visible device", device_mask);
  // A process that exits without nwc_shutdown (a Python caller, a node killed by its runtime)
  // still releases every device object of the library -- streams synchronised, copies finished,
  // pinned stages and HBM freed -- before the HIP runtime's own exit-time teardown: atexit
  // handlers run in reverse order of registration, and this one is registered after the runtime
  // was initialised above.  nwc_shutdown is idempotent (the second call finds no context).
  static const bool at_exit = std::atexit([] { nwc_shutdown(); }) == 0;
  (void)at_exit;
  // Test hook: NWC_VIRTUAL_DEVICES=k opens k contexts (own stream, tables, buffers) on a single
  // selected GPU, so the multi-device host paths -- shard threads, certificate cuts, bitmap
  // merges -- run for real on a one-GPU box (tests/test_gpu_multidev.py).
  const char* ve = std::getenv("NWC_VIRTUAL_DEVICES");
  const int virt = ve ? std::atoi(ve) : 0;
  const bool single = g_devs.size() == 1;
  for (int k = 1; single && k < virt && k < 32; ++k) {
    auto d = std::make_unique<DevCtx>();
    d->hip_id = g_devs[0]->hip_id;
    if (int rc = init_device(*d)) { g_devs.clear(); return rc; }
    g_devs.push_back(std::move(d));
  }
  return 0;
}

void nwc_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& d : g_devs) {
    std::lock_guard<std::mutex> dl(d->mu);
    (void)hipSetDevice(d->hip_id);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    if (d->arena) (void)hipFree(d->arena);
    if (d->scratch) (void)hipFree(d->scratch);
    if (d->fb_list) (void)hipFree(d->fb_list);
    if (d->fb_count) (void)hipFree(d->fb_count);
    if (d->pair_buf) (void)hipFree(d->pair_buf);
    if (d->sign_buf) (void)hipFree(d->sign_buf);
    if (d->stamps) (void)hipFree(d->stamps);
    if (d->cm_keys) (void)hipFree(d->cm_keys);
    if (d->cm_flags) (void)hipFree(d->cm_flags);
    if (d->cm_tables) (void)hipFree(d->cm_tables);
    if (d->cm_slots) (void)hipFree(d->cm_slots);
    if (d->cm_comb) (void)hipFree(d->cm_comb);
    if (d->ak_keys) (void)hipFree(d->ak_keys);
    if (d->ak_flags) (void)hipFree(d->ak_flags);
    if (d->ak_tables) (void)hipFree(d->ak_tables);
    if (d->ak_comb) (void)hipFree(d->ak_comb);
    if (d->ak_slots) (void)hipFree(d->ak_slots);
    if (d->comb_base) (void)hipFree(d->comb_base);
    if (d->base_table) (void)hipFree(d->base_table);
    if (d->base24) (void)hipFree(d->base24);
    if (d->base24_points) (void)hipFree(d->base24_points);
    if (d->km_keys) (void)hipFree(d->km_keys);
    if (d->km_flag) (void)hipFree(d->km_flag);
    if (d->comb16) (void)hipFree(d->comb16);
    if (d->comb16_bases) (void)hipFree(d->comb16_bases);
    if (d->kb_bases) (void)hipFree(d->kb_bases);
    if (d->straus_scratch) (void)hipFree(d->straus_scratch);
    if (d->msm_scratch) (void)hipFree(d->msm_scratch);
    if (d->rs_buf) (void)hipFree(d->rs_buf);
    if (d->msm_stats) (void)hipFree(d->msm_stats);
    if (d->lk_demand) (void)hipHostFree(d->lk_demand);
    if (d->lk_alloc) {
      (void)hipFree(d->lk.keys);
      (void)hipFree(d->lk.flags);
      (void)hipFree(d->lk.slots);
      (void)hipFree(d->lk.comb);
      (void)hipFree(d->lk.bases);
      (void)hipFree(d->lk.state);
    }
    if (d->pinned) (void)hipHostFree(d->pinned);
    if (d->cc_stakes) (void)hipFree(d->cc_stakes);
    if (d->cc_worker_off) (void)hipFree(d->cc_worker_off);
    if (d->cc_worker_ids) (void)hipFree(d->cc_worker_ids);
    if (d->msg_arena) (void)hipFree(d->msg_arena);
    if (d->uc_list) (void)hipFree(d->uc_list);
    if (d->uc_count) (void)hipFree(d->uc_count);
    if (d->ts_slots) (void)hipFree(d->ts_slots);
    if (d->ts_flag) (void)hipFree(d->ts_flag);
    if (d->ts_uniq) (void)hipFree(d->ts_uniq);
    if (d->ts_nuniq) (void)hipFree(d->ts_nuniq);
    if (d->km_keys) (void)hipFree(d->km_keys);
    if (d->km_flag) (void)hipFree(d->km_flag);
    if (d->scratch_free) (void)hipEventDestroy(d->scratch_free);
    if (d->base_table) (void)hipFree(d->base_table);
    if (d->base24) (void)hipFree(d->base24);
    if (d->base24_points) (void)hipFree(d->base24_points);
    if (d->side) (void)hipStreamSynchronize(d->side);
    if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
    if (d->ev_join) (void)hipEventDestroy(d->ev_join);
    if (d->ev_msg) (void)hipEventDestroy(d->ev_msg);
    if (d->ev_count) (void)hipEventDestroy(d->ev_count);
    if (d->side) (void)hipStreamDestroy(d->side);
    if (d->xfer) (void)hipStreamSynchronize(d->xfer);
    if (d->stager) d->stager->release();
    d->stager.reset();
    for (hipEvent_t e : d->ev_chunk) (void)hipEventDestroy(e);
    for (hipEvent_t e : d->ev_cnt) (void)hipEventDestroy(e);
    if (d->xfer) (void)hipStreamDestroy(d->xfer);
    if (d->stream) (void)hipStreamDestroy(d->stream);
  }
  g_devs.clear();
}

int nwc_device_count(void) { return (int)g_devs.size(); }

int nwc_verify_strict_many(const uint8_t* msgs32, const uint8_t* pks, const uint8_t* sigs, size_t n,
                           uint8_t* verdict_bitmap) {
  if (int rc = require_init()) return rc;
  if (n && (!msgs32 || !pks || !sigs || !verdict_bitmap)) return set_err(NWC_ERR_ARG, "null buffer");
  // per-device verdict words are merged into the caller's bitmap on this thread, after the join
  std::vector<std::vector<uint64_t>> parts(g_devs.size());
  std::vector<std::pair<uint64_t, uint64_t>> range(g_devs.size(), {0, 0});
  if (int rc = shard(n, [&](int di, uint64_t lo, uint64_t hi) -> int {
        range[di] = {lo, hi};
        return verify_range(di, msgs32, 1, nullptr, pks, sigs, lo, hi, 1, parts[di], 0);
      }))
    return rc;
  for (size_t di = 0; di < parts.size(); ++di)
    if (range[di].second > range[di].first) merge_bits(verdict_bitmap, range[di].first, parts[di], range[di].second - range[di].first);
  return 0;
}

int nwc_verify_strict(const uint8_t msg32[32], const uint8_t pk[32], const uint8_t sig[64]) {
  uint8_t bit = 0;
  int rc = nwc_verify_strict_many(msg32, pk, sig, 1, &bit);
  if (rc < 0) return rc;
  return (bit & 1) ? NWC_OK : NWC_INVALID;
}

int nwc_verify_batch(const uint8_t msg32[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                     uint8_t* bad_bitmap) {
  if (int rc = require_init()) return rc;
  if (n == 0) return NWC_OK;  // empty iterator: dalek verify_batch of nothing is Ok
  if (!msg32 || !pks || !sigs) return set_err(NWC_ERR_ARG, "null buffer");
  std::vector<uint64_t> words;
  if (int rc = verify_range(t_dev < (int)g_devs.size() ? t_dev : 0, msg32, 0, nullptr, pks, sigs, 0, n, 0, words, 0))
    return rc;
  bool all = true;
  for (size_t i = 0; i < n; ++i) all = all && ((words[i >> 6] >> (i & 63)) & 1);
  if (bad_bitmap) {
    std::vector<uint64_t> bad(words.size());
    for (size_t w = 0; w < words.size(); ++w) bad[w] = ~words[w];
    merge_bits(bad_bitmap, 0, bad, n);
  }
  return all ? NWC_OK : NWC_INVALID;
}

int nwc_verify_batch_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks, const uint8_t* sigs,
                          size_t m, uint8_t* cert_ok_bitmap, uint8_t* bad_vote_bitmap) {
  if (int rc = require_init()) return rc;
  if (m == 0) return 0;
  if (!digests || !offsets || !cert_ok_bitmap) return set_err(NWC_ERR_ARG, "null buffer");
  if (offsets[0] != 0) return set_err(NWC_ERR_ARG, "offsets[0] must be 0");
  for (size_t c = 0; c < m; ++c)
    if (offsets[c + 1] < offsets[c]) return set_err(NWC_ERR_ARG, "offsets not monotone at %zu", c);
  const uint64_t nv = offsets[m];
  if (nv && (!pks || !sigs)) return set_err(NWC_ERR_ARG, "null vote buffer");
  // the vote -> certificate index is built per device range (k_cert_index; on the host for small calls)
  using clk = std::chrono::steady_clock;
  const auto t1 = clk::now();
  // shard votes on certificate boundaries
  const int nd = (int)g_devs.size();
  std::vector<uint64_t> cuts(nd + 1);
  nwc_cert_cuts(offsets, m, (uint32_t)nd, cuts.data());
  std::vector<int> rc(nd, 0);
  std::vector<std::vector<uint64_t>> parts(nd);
  std::vector<std::thread> th;
  for (int i = 0; i < nd; ++i) {
    th.emplace_back([&, i] {
      rc[i] = verify_range(i, digests, 0, offsets, pks, sigs, cuts[i], cuts[i + 1], 0, parts[i], m);
    });
  }
  for (auto& t : th) t.join();
  for (int r : rc) if (r < 0) return r;
  const auto t2 = clk::now();
  const int r = batch_verdicts(offsets, m, cuts, parts, cert_ok_bitmap, bad_vote_bitmap);
  if (host_timing()) {
    auto ms = [](clk::duration d) { return std::chrono::duration<double>(d).count() * 1e3; };
    std::fprintf(stderr, "nwc_verify_batch_many: %zu certificates, %llu votes: devices %.2f ms, verdicts %.2f ms\n",
                 m, (unsigned long long)nv, ms(t2 - t1), ms(clk::now() - t2));
  }
  return r;
}

static int batch_equation_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks, const uint8_t* sigs,
                               size_t m, uint8_t* cert_ok_bitmap, uint8_t* bad_vote_bitmap, bool msm);

int nwc_verify_batch_straus_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks,
                                 const uint8_t* sigs, size_t m, uint8_t* cert_ok_bitmap, uint8_t* bad_vote_bitmap) {
  return batch_equation_many(digests, offsets, pks, sigs, m, cert_ok_bitmap, bad_vote_bitmap, false);
}

int nwc_verify_batch_msm_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks,
                              const uint8_t* sigs, size_t m, uint8_t* cert_ok_bitmap, uint8_t* bad_vote_bitmap) {
  return batch_equation_many(digests, offsets, pks, sigs, m, cert_ok_bitmap, bad_vote_bitmap, true);
}

static int batch_equation_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks, const uint8_t* sigs,
                               size_t m, uint8_t* cert_ok_bitmap, uint8_t* bad_vote_bitmap, bool msm) {
  if (int rc = require_init()) return rc;
  if (m == 0) return 0;
  if (!digests || !offsets || !cert_ok_bitmap) return set_err(NWC_ERR_ARG, "null buffer");
  if (offsets[0] != 0) return set_err(NWC_ERR_ARG, "offsets[0] must be 0");
  for (size_t c = 0; c < m; ++c)
    if (offsets[c + 1] < offsets[c]) return set_err(NWC_ERR_ARG, "offsets not monotone at %zu", c);
  const uint64_t nv = offsets[m];
  if (nv && (!pks || !sigs)) return set_err(NWC_ERR_ARG, "null vote buffer");
  const int nd = (int)g_devs.size();
  std::vector<uint64_t> cuts(nd + 1);
  nwc_cert_cuts(offsets, m, (uint32_t)nd, cuts.data());
  std::vector<int> rc(nd, 0);
  std::vector<std::vector<uint64_t>> parts(nd);
  std::vector<std::thread> th;
  for (int i = 0; i < nd; ++i)
    th.emplace_back([&, i] { rc[i] = straus_range(i, digests, m, offsets, pks, sigs, cuts[i], cuts[i + 1], parts[i], msm); });
  for (auto& t : th) t.join();
  for (int r : rc) if (r < 0) return r;
  return batch_verdicts(offsets, m, cuts, parts, cert_ok_bitmap, bad_vote_bitmap);
}

// Committee updates are serialised: the devices' caches and the host's view of them (g_hcm, which
// the latency path trusts) change together, one committee at a time.
std::mutex g_cm_mu;
static int set_committee_locked(const uint8_t* pks, size_t n);

// The committee cache holds exactly nwc_set_committee_config's committee (set there, cleared by
// nwc_set_committee): the message pipeline may then leave the strict equations of uncached keys
// undecided -- their authors are outside the committee, and UnknownAuthority precedes
// InvalidSignature for every message kind (primary/src/core.rs, messages.rs).
std::atomic<bool> g_cm_is_config{false};

int nwc_set_committee(const uint8_t* pks, size_t n) {
  std::lock_guard<std::mutex> lk(g_cm_mu);
  g_cm_is_config = false;
  return set_committee_locked(pks, n);
}

static int set_committee_locked(const uint8_t* pks, size_t n) {
  if (int rc = require_init()) return rc;
  if (n && !pks) return set_err(NWC_ERR_ARG, "null buffer");
  if (n > (1u << 20)) return set_err(NWC_ERR_ARG, "committee of %zu keys is too large", n);
  // open-addressing table (exact 32-byte keys), load factor <= 1/4, probe length bounded
  std::vector<nwc::u32> keys(8 * n);
  std::memcpy(keys.data(), pks, 32 * n);
  std::vector<int32_t> table;
  const uint32_t slots = build_slots(keys, n, table);
  {
    // host view cleared while the devices change (a call in between takes the general path),
    // set again once every device holds the new cache (end of this function)
    std::lock_guard<std::mutex> lk(g_hcm.mu);
    g_hcm.idx.slots.clear();
  }
  for (auto& dp : g_devs) {
    DevCtx& d = *dp;
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(hipEventSynchronize(d.scratch_free));   // no verify launch still reads the old cache
    HIP_TRY(hipStreamSynchronize(d.stream));
    auto_reset(d);   // keys remembered under the old committee are stale
    if (d.lk_alloc) {   // so are the launch keys (the next launch-key launch measures its demand anew)
      HIP_TRY(hipMemsetAsync(d.lk.slots, 0xFF, 4 * (size_t)nwc::LK_SLOTS, d.stream));
      HIP_TRY(hipMemsetAsync(d.lk.state, 0, 16, d.stream));
      d.lk_censused = false;
    }
    if (d.cm_keys) HIP_TRY(hipFree(d.cm_keys));
    if (d.cm_flags) HIP_TRY(hipFree(d.cm_flags));
    if (d.cm_tables) HIP_TRY(hipFree(d.cm_tables));
    if (d.cm_slots) HIP_TRY(hipFree(d.cm_slots));
    if (d.cm_comb) HIP_TRY(hipFree(d.cm_comb));
    d.cm_keys = nullptr; d.cm_flags = nullptr; d.cm_tables = nullptr; d.cm_slots = nullptr; d.cm_comb = nullptr;
    // stake / worker tables are indexed like the cache: a new cache invalidates them
    // (nwc_set_committee_config sets them again right after)
    if (d.cc_stakes) HIP_TRY(hipFree(d.cc_stakes));
    if (d.cc_worker_off) HIP_TRY(hipFree(d.cc_worker_off));
    if (d.cc_worker_ids) HIP_TRY(hipFree(d.cc_worker_ids));
    d.cc_stakes = nullptr; d.cc_worker_off = nullptr; d.cc_worker_ids = nullptr; d.cc_n = 0;
    d.cm_n = 0; d.cm_slot_mask = 0; d.cm_bytes = 0;
    if (n == 0) continue;
    HIP_TRY(hipMalloc(&d.cm_keys, 32 * n));
    HIP_TRY(hipMalloc(&d.cm_flags, 4 * n));
    HIP_TRY(hipMalloc(&d.cm_tables, n * 129 * sizeof(nwc::ge_niels)));
    HIP_TRY(hipMalloc(&d.cm_slots, 4 * (size_t)slots));
    HIP_TRY(hipMemcpyAsync(d.cm_keys, keys.data(), 32 * n, hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(d.cm_slots, table.data(), 4 * (size_t)slots, hipMemcpyHostToDevice, d.stream));
    const unsigned grid = (unsigned)((n * 129 + 255) / 256);
    hipLaunchKernelGGL(nwc::k_build_key_tables, dim3(grid), dim3(256), 0, d.stream, d.cm_keys, (nwc::u32)n,
                       d.cm_tables, d.cm_flags);
    HIP_TRY(hipGetLastError());
    if (n <= NWC_COMB_MAX_KEYS) {
      // per-key combs for the doubling-free path (radix 2^14: 20 MB per key)
      const size_t entries = n * nwc::COMB_PER_KEY;
      HIP_TRY(hipMalloc(&d.cm_comb, entries * sizeof(nwc::ge_niels_pad)));
      if (int rc = build_key_combs(d, d.cm_keys, (uint32_t)n, d.cm_comb)) return rc;
    }
    HIP_TRY(hipStreamSynchronize(d.stream));
    d.cm_n = (uint32_t)n;
    d.cm_slot_mask = slots - 1;
    d.cm_bytes = 36 * n + n * 129 * sizeof(nwc::ge_niels) + 4 * (size_t)slots +
                 (d.cm_comb ? n * nwc::COMB_PER_KEY * sizeof(nwc::ge_niels_pad) : 0);
  }
  if (n) {
    std::lock_guard<std::mutex> lk(g_hcm.mu);
    g_hcm.idx.keys = keys;
    g_hcm.idx.slots = table;
    g_hcm.idx.mask = slots - 1;
  }
  return 0;
}

int nwc_cache_stats(uint32_t* committee_keys, uint32_t* auto_keys) {
  if (int rc = require_init()) return rc;
  DevCtx& d = *ctx(t_dev < (int)g_devs.size() ? t_dev : 0);
  std::lock_guard<std::mutex> lk(d.mu);
  if (committee_keys) *committee_keys = d.cm_n;
  if (auto_keys) *auto_keys = d.ak_n;
  return 0;
}

int nwc_launch_keys_info(uint32_t* held, uint32_t* capacity) {
  if (int rc = require_init()) return rc;
  DevCtx& d = *ctx(t_dev < (int)g_devs.size() ? t_dev : 0);
  std::lock_guard<std::mutex> g(d.mu);
  uint32_t st[4] = {0, 0, 0, 0};
  if (d.lk_alloc) {
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(hipDeviceSynchronize());   // the set is updated on callers' streams
    HIP_TRY(hipMemcpy(st, d.lk.state, 16, hipMemcpyDeviceToHost));
  }
  if (held) *held = st[0];
  if (capacity) *capacity = nwc::LK_MAX_KEYS;
  return 0;
}

int nwc_auto_cache_info(uint32_t* capacity, uint64_t* builds, uint64_t* hits) {
  if (int rc = require_init()) return rc;
  DevCtx& d = *ctx(t_dev < (int)g_devs.size() ? t_dev : 0);
  std::lock_guard<std::mutex> lk(d.mu);
  if (capacity) *capacity = auto_keys_cap();
  if (builds) *builds = d.ak_builds;
  if (hits) *hits = d.ak_hits;
  return 0;
}

int nwc_sha512_trunc32_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32) {
  if (int rc = require_init()) return rc;
  if (n == 0) return 0;
  if (!offsets || !out32) return set_err(NWC_ERR_ARG, "null buffer");
  for (size_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return set_err(NWC_ERR_ARG, "offsets not monotone at %zu", i);
  if (offsets[n] > offsets[0] && !data) return set_err(NWC_ERR_ARG, "null data");
  return shard(n, [&](int di, uint64_t lo, uint64_t hi) -> int {
    DevCtx& d = *ctx(di);
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.hip_id));
    const uint64_t k = hi - lo;
    if (k == 0) return 0;
    // Device layout: every message starts 16-byte aligned (the kernel's dwordx4 path).
    std::vector<uint64_t> starts(k), ends(k);
    uint64_t total = 0;
    for (uint64_t i = 0; i < k; ++i) {
      const uint64_t len = offsets[lo + i + 1] - offsets[lo + i];
      starts[i] = total;
      ends[i] = total + len;
      total += (len + 15) & ~15ull;
    }
    const size_t need = align256(total + 16) + 2 * align256(8 * k) + align256(32 * k);
    if (int rc = d.ensure_arena(need)) return rc;
    Carve c(d.arena);
    uint8_t* dd = c.take<uint8_t>(total + 16);
    uint64_t* dstarts = c.take<uint64_t>(8 * k);
    uint64_t* dends = c.take<uint64_t>(8 * k);
    uint8_t* dout = c.take<uint8_t>(32 * k);
    const bool aligned = (offsets[lo] % 16 == 0) && [&] {
      for (uint64_t i = 0; i < k; ++i) if (offsets[lo + i] - offsets[lo] != starts[i]) return false;
      return true;
    }();
    if (aligned) {
      if (total) HIP_TRY(hipMemcpyAsync(dd, data + offsets[lo], offsets[hi] - offsets[lo], hipMemcpyHostToDevice, d.stream));
    } else {
      std::vector<uint8_t> stage(total);
      for (uint64_t i = 0; i < k; ++i)
        if (ends[i] > starts[i]) std::memcpy(stage.data() + starts[i], data + offsets[lo + i], ends[i] - starts[i]);
      if (total) HIP_TRY(hipMemcpyAsync(dd, stage.data(), total, hipMemcpyHostToDevice, d.stream));
      HIP_TRY(hipStreamSynchronize(d.stream));  // `stage` is pageable and about to go out of scope
    }
    HIP_TRY(hipMemcpyAsync(dstarts, starts.data(), 8 * k, hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(dends, ends.data(), 8 * k, hipMemcpyHostToDevice, d.stream));
    if (int rc = launch_digest(dd, dstarts, dends, k, dout, d.stream)) return rc;
    HIP_TRY(hipMemcpyAsync(out32 + 32 * lo, dout, 32 * k, hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    return 0;
  });
}

int nwc_digest32(const uint8_t* data, size_t len, uint8_t out32[32]) {
  uint64_t offs[2] = {0, (uint64_t)len};
  return nwc_sha512_trunc32_many(data, offs, 1, out32);
}

// ---- device-resident ---------------------------------------------------------------------
int nwc_dev_set_device(int device) {
  if (int rc = require_init()) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return set_err(NWC_ERR_ARG, "device %d not initialised", device);
  t_dev = device;
  return 0;
}

#define DEV_PROLOGUE                                                        \
  if (int rc_ = require_init()) return rc_;                                 \
  DevCtx& d = *ctx(t_dev < (int)g_devs.size() ? t_dev : 0);                 \
  std::lock_guard<std::mutex> lk(d.mu);                                     \
  HIP_TRY(hipSetDevice(d.hip_id));                                          \
  hipStream_t s = reinterpret_cast<hipStream_t>(stream); /* NULL = HIP default stream */

int nwc_dev_verify(const void* d_msgs, const void* d_msg_index, uint64_t msg_stride, const void* d_pks,
                   const void* d_sigs, uint64_t n, int strict, void* d_verdict_words, void* stream) {
  DEV_PROLOGUE
  if (n && (!d_msgs || !d_pks || !d_sigs || !d_verdict_words)) return set_err(NWC_ERR_ARG, "null buffer");
  return launch_verify(d, (const uint8_t*)d_msgs, (const uint32_t*)d_msg_index, msg_stride, (const uint8_t*)d_pks,
                       (const uint8_t*)d_sigs, n, strict, (uint64_t*)d_verdict_words, s);
}

int nwc_diag_verify_clock(const void* d_msgs, uint64_t msg_stride, const void* d_pks, const void* d_sigs, uint64_t n,
                          void* d_verdict_words, void* stream, double* clock_ghz, uint32_t* waves) {
  DEV_PROLOGUE
  if (!d_msgs || !d_pks || !d_sigs || !d_verdict_words || !clock_ghz) return set_err(NWC_ERR_ARG, "null buffer");
  if (n < 4096) return set_err(NWC_ERR_ARG, "the clock stamp needs a full launch (n >= 4096)");
  // the stamps come from the plain k_verify launch: a committee cache would send these strict
  // equations to the comb kernel (no stamps), and a split launch would overwrite them
  if (d.cm_n) return set_err(NWC_ERR_ARG, "the clock stamp needs the plain k_verify path: clear the committee cache first");
  if (n > verify_max_launch())
    return set_err(NWC_ERR_ARG, "the clock stamp needs a single launch (n <= %llu)", (unsigned long long)verify_max_launch());
  // one stamp slot per wave of the largest grid launch_verify gives k_verify
  const uint64_t nwaves = (uint64_t)d.cus * d.verify_blocks_per_cu * NWC_VERIFY_GRID_MULT * 4;
  if (!d.stamps) HIP_TRY(hipMalloc(&d.stamps, 32 * nwaves));
  HIP_TRY(hipMemsetAsync(d.stamps, 0, 32 * nwaves, s));
  if (int rc = launch_verify(d, (const uint8_t*)d_msgs, nullptr, msg_stride, (const uint8_t*)d_pks, (const uint8_t*)d_sigs,
                             n, 1, (uint64_t*)d_verdict_words, s, LV_STAMP))
    return rc;
  std::vector<uint64_t> st(4 * nwaves);
  HIP_TRY(hipMemcpyAsync(st.data(), d.stamps, 32 * nwaves, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::vector<double> ghz;
  for (uint64_t w = 0; w < nwaves; ++w) {
    const uint64_t* x = &st[4 * w];
    // a wave that ran at least ~10 us of real time (100 MHz ticks)
    if (x[3] > x[2] + 1000 && x[1] > x[0]) ghz.push_back((double)(x[1] - x[0]) / (double)(x[3] - x[2]) * 0.1);
  }
  if (ghz.empty()) return set_err(NWC_ERR_DEVICE, "no wave stamped its clock");
  std::nth_element(ghz.begin(), ghz.begin() + ghz.size() / 2, ghz.end());
  *clock_ghz = ghz[ghz.size() / 2];
  if (waves) *waves = (uint32_t)ghz.size();
  return 0;
}

int nwc_dev_cert_reduce(const void* d_leaf_words, const void* d_offsets, uint64_t m, uint64_t nvotes,
                        void* d_cert_words, void* d_bad_words, void* stream) {
  DEV_PROLOGUE
  return launch_cert_reduce((const uint64_t*)d_leaf_words, (const uint32_t*)d_offsets, m, nvotes,
                            (uint64_t*)d_cert_words, (uint64_t*)d_bad_words, s);
}

int nwc_dev_verify_batch_straus(const void* d_digests, const void* d_offsets, const void* d_msg_index, uint64_t m,
                                uint64_t nvotes, const void* d_pks, const void* d_sigs, void* d_leaf_words,
                                void* stream) {
  DEV_PROLOGUE
  if (m == 0 || nvotes == 0) return 0;
  if (!d_digests || !d_offsets || !d_msg_index || !d_pks || !d_sigs || !d_leaf_words)
    return set_err(NWC_ERR_ARG, "null buffer");
  return launch_straus(d, static_cast<const uint8_t*>(d_digests), static_cast<const uint32_t*>(d_msg_index),
                       static_cast<const uint8_t*>(d_pks), static_cast<const uint8_t*>(d_sigs), nvotes,
                       static_cast<uint64_t*>(d_leaf_words), s);
}

int nwc_dev_verify_batch_msm(const void* d_digests, const void* d_offsets, const void* d_msg_index, uint64_t m,
                             uint64_t nvotes, const void* d_pks, const void* d_sigs, void* d_leaf_words, void* stream) {
  DEV_PROLOGUE
  if (m == 0 || nvotes == 0) return 0;
  if (!d_digests || !d_offsets || !d_msg_index || !d_pks || !d_sigs || !d_leaf_words)
    return set_err(NWC_ERR_ARG, "null buffer");
  return launch_batch_dalek(d, static_cast<const uint8_t*>(d_digests), static_cast<const uint32_t*>(d_msg_index), m,
                            static_cast<const uint8_t*>(d_pks), static_cast<const uint8_t*>(d_sigs), nvotes,
                            static_cast<uint64_t*>(d_leaf_words), s);
}

int nwc_msm_stats(uint64_t* groups_passed, uint64_t* groups_failed, uint64_t* key_overflows, uint64_t* groups_skipped) {
  if (int rc = require_init()) return rc;
  DevCtx* dp = ctx(t_dev);
  if (!dp) return set_err(NWC_ERR_ARG, "device index %d not initialised", t_dev);
  DevCtx& d = *dp;
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.hip_id));
  uint32_t st[nwc::MSM_ST_WORDS] = {};
  if (d.msm_stats) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(st, d.msm_stats, sizeof st, hipMemcpyDeviceToHost));
  }
  if (groups_passed) *groups_passed = st[nwc::MSM_ST_PASSED];
  if (groups_failed) *groups_failed = st[nwc::MSM_ST_FAILED];
  if (key_overflows) *key_overflows = st[nwc::MSM_ST_OVERFLOW];
  if (groups_skipped) *groups_skipped = st[nwc::MSM_ST_SKIPPED];
  return 0;
}

int nwc_dev_sha512_trunc32(const void* d_data, const void* d_offsets, uint64_t n, void* d_out32, void* stream) {
  DEV_PROLOGUE
  return launch_digest((const uint8_t*)d_data, (const uint64_t*)d_offsets, nullptr, n, (uint8_t*)d_out32, s);
}

int nwc_dev_sha512_trunc32_ranges(const void* d_data, const void* d_starts, const void* d_ends, uint64_t n,
                                  void* d_out32, void* stream) {
  DEV_PROLOGUE
  if (n && (!d_starts || !d_ends || !d_out32)) return set_err(NWC_ERR_ARG, "null buffer");
  return launch_digest((const uint8_t*)d_data, (const uint64_t*)d_starts, (const uint64_t*)d_ends, n,
                       (uint8_t*)d_out32, s);
}

int nwc_dev_derive32(const uint8_t* tag, int taglen, uint64_t first, uint64_t n, void* d_out, void* stream) {
  DEV_PROLOGUE
  if (taglen < 0 || taglen > 96) return set_err(NWC_ERR_ARG, "tag longer than 96 bytes");
  if (n == 0) return 0;
  nwc::Tag64 t;
  std::memset(&t, 0, sizeof t);
  if (taglen > 64) return set_err(NWC_ERR_ARG, "tag longer than 64 bytes");
  std::memcpy(t.b, tag, (size_t)taglen);
  hipLaunchKernelGGL(nwc::k_derive32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, t, taglen, first, n,
                     (uint8_t*)d_out);
  HIP_TRY(hipGetLastError());
  return 0;
}

int nwc_dev_keygen_sign(const void* d_seeds, const void* d_msgs, uint64_t n, void* d_pks, void* d_sigs,
                        void* stream) {
  DEV_PROLOGUE
  if (n == 0) return 0;
  if (int rc = ensure_verify_tables(d)) return rc;
  hipLaunchKernelGGL(nwc::k_keygen_sign, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const uint8_t*)d_seeds,
                     (const uint8_t*)d_msgs, n, (uint8_t*)d_pks, (uint8_t*)d_sigs, d.base_table);
  HIP_TRY(hipGetLastError());
  return 0;
}


int nwc_set_committee_config(const uint8_t* pks, const uint64_t* stakes, size_t n, const uint32_t* worker_offsets,
                             const uint32_t* worker_ids) {
  if (int rc = require_init()) return rc;
  if (n && (!pks || !stakes || !worker_offsets)) return set_err(NWC_ERR_ARG, "null buffer");
  if (n && worker_offsets[0] != 0) return set_err(NWC_ERR_ARG, "worker_offsets[0] must be 0");
  if (n > nwc::MSG_MAX_COMMITTEE)
    return set_err(NWC_ERR_ARG, "committee of %zu authorities exceeds %u", n, nwc::MSG_MAX_COMMITTEE);
  for (size_t k = 0; k < n; ++k)
    if (worker_offsets[k + 1] < worker_offsets[k]) return set_err(NWC_ERR_ARG, "worker_offsets not monotone");
  const uint32_t nw = n ? worker_offsets[n] : 0;
  if (nw && !worker_ids) return set_err(NWC_ERR_ARG, "null worker ids");
  // config::Committee holds a BTreeMap<PublicKey, Authority>: a key listed twice is one authority
  // with the LAST entry's stake and workers (a map insert replaces the value).  Deduplicate so the
  // cache index, the stake table and the quorum (config/src/lib.rs:181-186) all see that map.
  std::vector<uint8_t> ukeys;
  std::vector<uint64_t> ustakes;
  std::vector<uint32_t> uoff{0}, uids;
  {
    std::vector<size_t> last;   // entry index of the last occurrence, in first-appearance order
    for (size_t k = 0; k < n; ++k) {
      size_t j = 0;
      while (j < last.size() && std::memcmp(pks + 32 * last[j], pks + 32 * k, 32) != 0) ++j;
      if (j == last.size()) last.push_back(k);
      else last[j] = k;
    }
    for (size_t k : last) {
      ukeys.insert(ukeys.end(), pks + 32 * k, pks + 32 * k + 32);
      ustakes.push_back(stakes[k]);
      if (worker_offsets[k + 1] > worker_offsets[k])
        uids.insert(uids.end(), worker_ids + worker_offsets[k], worker_ids + worker_offsets[k + 1]);
      uoff.push_back((uint32_t)uids.size());
    }
  }
  n = ustakes.size();
  pks = ukeys.data();
  stakes = ustakes.data();
  worker_offsets = uoff.data();
  worker_ids = uids.data();
  std::lock_guard<std::mutex> cm_lk(g_cm_mu);
  g_cm_is_config = false;
  if (int rc = set_committee_locked(pks, n)) return rc;
  g_cm_is_config = true;
  uint64_t total = 0;
  for (size_t k = 0; k < n; ++k) total += stakes[k];
  for (auto& dp : g_devs) {
    DevCtx& d = *dp;
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(hipStreamSynchronize(d.stream));
    if (d.cc_stakes) HIP_TRY(hipFree(d.cc_stakes));
    if (d.cc_worker_off) HIP_TRY(hipFree(d.cc_worker_off));
    if (d.cc_worker_ids) HIP_TRY(hipFree(d.cc_worker_ids));
    d.cc_stakes = nullptr; d.cc_worker_off = nullptr; d.cc_worker_ids = nullptr;
    d.cc_n = 0;
    d.cc_quorum = 2 * total / 3 + 1;   // Committee::quorum_threshold (config/src/lib.rs:168-173)
    HIP_TRY(hipMalloc(&d.cc_stakes, 8 * (n + 1)));
    HIP_TRY(hipMalloc(&d.cc_worker_off, 4 * (n + 1)));
    HIP_TRY(hipMalloc(&d.cc_worker_ids, 4 * (size_t)(nw + 1)));
    if (n) {
      HIP_TRY(hipMemcpy(d.cc_stakes, stakes, 8 * n, hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(d.cc_worker_off, worker_offsets, 4 * (n + 1), hipMemcpyHostToDevice));
      if (!uids.empty()) HIP_TRY(hipMemcpy(d.cc_worker_ids, worker_ids, 4 * uids.size(), hipMemcpyHostToDevice));
    }
    d.cc_n = (uint32_t)n;
  }
  return 0;
}

// Device part of nwc_sanitize_messages: messages in HBM (ddata 4-byte aligned with >= 16 bytes
// of readable padding, doff device u64[m+1] relative to ddata, `total` bytes), parsed as the
// chunks cuts[k] .. cuts[k+1] (whole messages).  `chunk_ready(k)`, when given, returns once chunk
// k's bytes are on their way and stream s waits for them (the host path's copies);
// `chunk_queued(k)` tells without waiting whether they are, and chunk k's parse is then queued
// before the host waits for chunk k - 1's count.  The chunks share one vote-slot counter, so the
// votes of the chunks parsed so far are contiguous; after each parse the host reads the count and
// launches those votes' leaves on the side stream beside the next chunk's parse, and the rest
// after the last chunk.  (Measured and removed in round 6: leaves behind the parses on one stream,
// leaves in whole comb rounds, per-launch list passes, each parse queued only after the previous
// count -- profiles/r05/wire_host.md, ab_wire_modes.txt, ab_wire_defer_lists.txt.)
// The strict equations (headers' and votes' own signatures) of all chunks but the last run while
// the last one crosses PCIe; the header digests and the final codes run once over all m messages.
static int sanitize_dev(DevCtx& d, const uint8_t* ddata, const uint64_t* doff, size_t m, uint64_t total,
                        const std::vector<size_t>& cuts, uint64_t gc_round, const uint8_t* vote_target, int32_t* dcodes,
                        uint8_t* ddigests, uint32_t* drec, hipStream_t s,
                        const std::function<int(size_t)>& chunk_ready = nullptr,
                        const std::function<bool(size_t)>& chunk_queued = nullptr) {
  if (int rc = ensure_verify_tables(d)) return rc;
  const size_t nch = cuts.size() - 1;
  // a vote list is allocated only when wholly inside its message (>= 72 B per vote)
  const uint64_t vt = total / 72 + 1 + (nch > 1 ? 64 * nch : 0);   // + the 64-slot alignment of each chunk
  if (vt > 0xFFFFFFFFull) return set_err(NWC_ERR_ARG, "too many vote slots in one call");
  // the leaf launches of a chunked call on the committee-cache comb path only list their uncached
  // equations (LV_DEFER_LIST); the list's half-size, fallback and torsion passes run once, after
  // the leaves queued before the first strict launch (which reuses the list), instead of ~8 small
  // launches per chunk on the leaf stream.  Their sign tests are deferred too (SignRecs,
  // k_verify_comb_y / k_comb_sign): a chunk's ~1 vote per lane would otherwise pay a whole
  // inversion per vote.  NWC_SIGN_DEFER=0: k_verify_comb per chunk (A/B).
  const bool chunked = nch > 1;
  const bool defer = chunked && deferrable_list(d);
  const bool ysplit = defer && sign_defer();
  const size_t need = align256(total + 128 * (m + 2)) + align256(32 * m) * 3 + align256(64 * m) + align256(32 * vt) +
                      align256(64 * vt) + align256(4 * vt) + align256(4) + align256(4 * m) + align256(16 * m) +
                      align256(4 * m) + align256(8 * ((m + 63) / 64)) + align256(8 * ((vt + 63) / 64)) +
                      (ysplit ? 3 * align256(32 * vt) + align256(4 * vt) + 3 * align256(32 * m) + align256(4 * m) : 0);
  if (need > d.msg_arena_cap) {
    HIP_TRY(hipEventSynchronize(d.scratch_free));
    HIP_TRY(hipStreamSynchronize(s));
    if (d.msg_arena) HIP_TRY(hipFree(d.msg_arena));
    d.msg_arena = nullptr;
    d.msg_arena_cap = 0;
    const size_t cap = need + need / 4 + (1 << 20);
    HIP_TRY(hipMalloc(&d.msg_arena, cap));
    d.msg_arena_cap = cap;
  }
  Carve c(d.msg_arena);
  nwc::MsgArgs a{};   // the whole call's arrays
  a.data = ddata;
  a.offsets = doff;
  a.m = m;
  a.gc_round = gc_round;
  a.hashbuf = c.take<uint8_t>(total + 128 * (m + 2));
  a.eq_msg = c.take<uint8_t>(32 * m);
  a.eq_pk = c.take<uint8_t>(32 * m);
  a.eq_sig = c.take<uint8_t>(64 * m);
  a.cdig = c.take<uint8_t>(32 * m);
  a.v_pk = c.take<uint8_t>(32 * vt);
  a.v_sig = c.take<uint8_t>(64 * vt);
  a.v_msg = c.take<uint32_t>(4 * vt);
  a.v_total = c.take<uint32_t>(4);
  a.v_cap = vt;
  a.hmatch = c.take<uint32_t>(4 * m);
  a.rec = drec ? drec : c.take<uint32_t>(16 * m);
  a.rec_n = c.take<uint32_t>(4 * m);
  uint64_t* sbits = c.take<uint64_t>(8 * ((m + 63) / 64));
  uint64_t* lbits = c.take<uint64_t>(8 * ((vt + 63) / 64));
  nwc::SignRecs sr{};   // vote v's record at index v
  if (ysplit) {
    sr.x = c.take<uint32_t>(32 * vt);
    sr.z = c.take<uint32_t>(32 * vt);
    sr.p = c.take<uint32_t>(32 * vt);
    sr.meta = c.take<uint32_t>(4 * vt);
    HIP_TRY(hipMemsetAsync(lbits, 0, 8 * ((vt + 63) / 64), s));   // the sign and list passes OR into it
  }
  nwc::SignRecs srs{};   // the strict equations' records (message i at index i)
  if (ysplit) {
    srs.x = c.take<uint32_t>(32 * m);
    srs.z = c.take<uint32_t>(32 * m);
    srs.p = c.take<uint32_t>(32 * m);
    srs.meta = c.take<uint32_t>(4 * m);
    HIP_TRY(hipMemsetAsync(sbits, 0, 8 * ((m + 63) / 64), s));
  }
  a.digests = ddigests;
  if (vote_target) {
    a.target.enabled = 1;
    std::memcpy(a.target.id, vote_target, 32);
    std::memcpy(&a.target.round, vote_target + 32, 8);
    std::memcpy(a.target.origin, vote_target + 40, 32);
  }
  if (int rc = d.ensure_pinned(NWC_PINNED_STAGE_MAX)) return rc;
  if (4 * nch > (64u << 10)) return set_err(NWC_ERR_ARG, "too many chunks");   // counts below sanitize_range's offsets
  uint32_t* nv_host = reinterpret_cast<uint32_t*>(d.pinned);   // pinned: the count copies stay asynchronous
  while (d.ev_cnt.size() < nch) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    d.ev_cnt.push_back(e);
  }
  // the leaf stream when chunks overlap: the side stream, which has a hardware queue of its own
  // (GPU_MAX_HW_QUEUES = 4: a stream created later shared the transfer stream's queue, and its
  // leaves waited behind the markers of the in-flight copies, profiles/r05/wire_host.md)
  const hipStream_t ls = chunked ? d.side : s;
  struct HoldLists {
    DevCtx& d;
    ~HoldLists() { d.hold_lists = false; }
  } hold{d};
  if (defer) {
    if (int rc = ensure_scratch(d, 0, vt)) return rc;
    d.hold_lists = true;
    HIP_TRY(hipStreamWaitEvent(ls, d.scratch_free, 0));
    HIP_TRY(hipMemsetAsync(d.uc_count, 0, sizeof(uint32_t), ls));
  }
  bool pending = false;   // deferred leaf launches whose list passes have not been queued
  HIP_TRY(hipMemsetAsync(a.v_total, 0, 4, s));
  HIP_TRY(hipMemsetAsync(a.v_msg, 0, 4 * vt, s));
  const nwc::Committee cm{d.cm_keys, d.cm_flags, d.cm_tables, d.cm_comb, d.cm_slots, d.cm_slot_mask, d.cm_n};
  const nwc::CommitteeCfg cc{d.cc_stakes, d.cc_worker_off, d.cc_worker_ids, d.cc_quorum, d.cc_n};
  const size_t first_lds = 4 * (size_t)std::max<uint32_t>(1, std::min<uint32_t>(d.cc_n, nwc::MSG_MAX_COMMITTEE));
  // NWC_HOST_TIMING: host-side stamps of the steps (which call waits on what)
  const bool timing = host_timing();
  const auto tm0 = std::chrono::steady_clock::now();
  std::vector<std::pair<const char*, double>> marks;
  auto mark = [&](const char* what) {
    if (timing) marks.emplace_back(what, std::chrono::duration<double>(std::chrono::steady_clock::now() - tm0).count() * 1e3);
  };
  uint64_t launched = 0;   // votes [0, launched) have their leaf launch queued
  bool list_dirty = false;   // a strict launch on ls has reused the uncached list since its reset
  // ysplit: votes [owed_lo, owed_hi) have had their leaves but not their sign tests yet; those run
  // in the first blocks of the next chunk's leaf launch (k_verify_comb_y_sign), so their
  // latency-bound chain overlaps its comb sums, or alone before a list pass needs their words
  uint64_t owed_lo = 0, owed_hi = 0;
  auto leaves = [&](uint64_t upto, bool deferred) -> int {
    if (upto <= launched) return 0;
    if (deferred && list_dirty) {
      HIP_TRY(hipMemsetAsync(d.uc_count, 0, sizeof(uint32_t), ls));
      list_dirty = false;
    }
    const uint64_t v0 = launched;
    const bool y = deferred && ysplit;
    const nwc::SignPass sp{sr, owed_lo, owed_hi - owed_lo, lbits, comb_sign_blocks(d, owed_hi - owed_lo)};
    const nwc::SignRecs srl = sign_recs_at(sr, (int64_t)v0);
    if (int rc = launch_verify(d, a.cdig, a.v_msg + v0, 0, a.v_pk + 32 * v0, a.v_sig + 64 * v0, upto - v0, 0,
                               lbits + v0 / 64, ls, deferred ? LV_DEFER_LIST : 0, nullptr, v0, nullptr,
                               y ? &srl : nullptr, y ? &sp : nullptr))
      return rc;
    if (y) {
      owed_lo = v0;
      owed_hi = upto;
    }
    pending = pending || deferred;
    launched = upto;
    mark("leaves queued");
    return 0;
  };
  // the list passes of the deferred leaves so far (they OR the uncached votes' bits into the words
  // the comb or sign kernels wrote), after the sign tests still owed
  auto finish = [&]() -> int {
    if (owed_hi > owed_lo) {
      if (int rc = launch_comb_sign(d, sr, owed_lo, owed_hi - owed_lo, lbits, ls)) return rc;
      owed_lo = owed_hi;
    }
    if (!pending) return 0;
    pending = false;
    return finish_deferred_list(d, a.cdig, a.v_msg, 0, a.v_pk, a.v_sig, launched, 0, lbits, ls);
  };
  // the strict equations (headers' and votes' own signatures) of messages [c0, c1) on the leaf
  // stream, after the list passes (the strict launch reuses the list)
  // With the cache holding exactly the configured committee (g_cm_is_config) and the sign tests
  // deferred, strict equations [c0, c1) go on the parse stream as k_verify_comb_y without a list
  // (an uncached key is a non-member: UnknownAuthority decides first) and their sign pass, off the
  // leaf stream, which then carries only the leaves and their list passes.
  bool strict_y = false;   // set below once the cuts are known to be aligned
  auto strict = [&](size_t c0, size_t c1) -> int {
    if (c1 <= c0) return 0;
    if (strict_y) {
      const uint64_t n = c1 - c0;
      const nwc::VerifyArgs va{a.eq_msg + 32 * c0, nullptr, 1, a.eq_pk + 32 * c0, a.eq_sig + 64 * c0, sbits + c0 / 64,
                               n, 1, d.base_table, d.base24, d.scratch, d.fb_list, d.fb_count, 0u, cm};
      const nwc::CombArgs ca{nullptr, nullptr, d.comb_base, d.comb16, nullptr, 0};
      const unsigned gy = (unsigned)std::min<uint64_t>((n + 255) / 256, 60000);
      hipLaunchKernelGGL(nwc::k_verify_comb_y, dim3(gy), dim3(256), 0, s, va, ca, sign_recs_at(srs, (int64_t)c0));
      HIP_TRY(hipGetLastError());
      return launch_comb_sign(d, srs, c0, n, sbits, s);
    }
    if (int rc = finish()) return rc;
    list_dirty = true;
    return launch_verify(d, a.eq_msg + 32 * c0, nullptr, 1, a.eq_pk + 32 * c0, a.eq_sig + 64 * c0, c1 - c0, 1,
                         sbits + c0 / 64, ls);
  };
  // The strict equations of the first chunks go in one launch after chunk strict_at's leaves,
  // early, where the leaf stream has slack to absorb its ~0.17 ms (a latency-bound launch); the
  // rest at the end (every cut is a multiple of 64 messages, sanitize_range: each strict launch
  // owns its verdict words).  (A strict launch per chunk, each after a list pass, measured 20 %
  // slower; at chunk nch - 3 instead of nch / 3, within noise: profiles/r06/wire_sign/.)
  bool aligned = true;
  for (size_t k = 1; k < nch; ++k) aligned = aligned && (cuts[k] & 63) == 0;
  const size_t strict_at = aligned && nch >= 3 ? nch / 3 : (nch >= 2 ? nch - 2 : 0);   // its iteration k
  strict_y = ysplit && aligned && g_cm_is_config.load() && strict_y_on();
  size_t strict_done = 0;   // messages [0, strict_done) have their strict launch queued
  uint64_t nv = 0;
  size_t queued = 0;   // chunks whose parse is queued
  auto queue_parse = [&]() -> int {
    const size_t k = queued++;
    if (chunk_ready)
      if (int rc = chunk_ready(k)) return rc;
    mark("chunk ready");
    const size_t c0 = cuts[k];
    nwc::MsgArgs ak = a;
    ak.offsets = doff + c0;
    ak.m = cuts[k + 1] - c0;
    ak.hashbuf = a.hashbuf + 128 * c0;   // the message's slot: aligned data offset + 128 x (call-wide index)
    ak.eq_msg = a.eq_msg + 32 * c0;
    ak.eq_pk = a.eq_pk + 32 * c0;
    ak.eq_sig = a.eq_sig + 64 * c0;
    ak.cdig = a.cdig + 32 * c0;
    ak.msg_base = (uint32_t)c0;
    ak.hmatch = a.hmatch + c0;
    ak.rec = a.rec + 4 * c0;
    ak.rec_n = a.rec_n + c0;
    ak.digests = ddigests ? ddigests + 32 * c0 : nullptr;
    hipLaunchKernelGGL(nwc::k_parse_messages, dim3((unsigned)ak.m), dim3(64), first_lds, s, ak, cm, cc);
    HIP_TRY(hipGetLastError());
    if (nch > 1) {
      // the next chunk's votes from a 64-slot boundary: every leaf launch starts on its own
      // verdict word (the skipped slots repeat the last vote; their leaves are never read)
      hipLaunchKernelGGL(nwc::k_align_slots, dim3(1), dim3(64), 0, s, a.v_total, (uint32_t)vt, a.v_pk, a.v_sig,
                         a.v_msg);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemcpyAsync(nv_host + k, a.v_total, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(d.ev_cnt[k], s));
    mark("parse queued");
    return 0;
  };
  if (int rc = queue_parse()) return rc;
  for (size_t k = 0; k < nch; ++k) {
    // the next chunk's parse goes in before this chunk's count is awaited when its copy is already
    // queued (no wait on the copier): it then follows this parse on the GPU without a host round
    // trip in between
    if (queued < nch && (!chunk_queued || chunk_queued(queued)))
      if (int rc = queue_parse()) return rc;
    if (!chunked) continue;
    // the votes parsed so far on the leaf stream; the next chunk's copy goes on in the copier
    // thread meanwhile, and its parse runs beside these leaves
    HIP_TRY(hipEventSynchronize(d.ev_cnt[k]));
    nv = std::min<uint64_t>(nv_host[k], vt);
    mark("count");
    HIP_TRY(hipStreamWaitEvent(ls, d.ev_cnt[k], 0));
    // (the last leaf launch then holds only the last chunk's votes)
    if (k + 1 < nch)
      if (int rc = leaves(nv, defer)) return rc;
    if (k == strict_at) {
      if (int rc = strict(0, cuts[k + 1])) return rc;
      strict_done = cuts[k + 1];
    }
    if (queued == k + 1 && queued < nch)
      if (int rc = queue_parse()) return rc;
  }
  if (chunked) {
    // the Header::digest checks once, beside the last leaves (latency-bound: ~0.2 ms for any
    // number of messages, so not per chunk)
    hipLaunchKernelGGL(nwc::k_header_digests, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, a);
    HIP_TRY(hipGetLastError());
    if (ysplit) {
      // the last chunk's leaves deferred as well (a fresh list: the strict launch reused it),
      // their sign tests, then the list passes and the remaining strict equations
      if (int rc = leaves(nv, true)) return rc;
      if (int rc = strict(strict_done, m)) return rc;
      if (int rc = finish()) return rc;   // (strict_y: the strict launches left the leaf stream's passes)
    } else {
      if (int rc = strict(strict_done, m)) return rc;
      if (int rc = leaves(nv, false)) return rc;
    }
    HIP_TRY(hipEventRecord(d.ev_msg, ls));
    HIP_TRY(hipStreamWaitEvent(s, d.ev_msg, 0));
  } else {
    // one chunk: the strict launch (it needs no count) queued before the host waits for the
    // count, the Header::digest checks beside the leaves on the side stream
    if (int rc = launch_verify(d, a.eq_msg, nullptr, 1, a.eq_pk, a.eq_sig, m, 1, sbits, s)) return rc;
    HIP_TRY(hipEventRecord(d.ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(d.side, d.ev_fork, 0));
    hipLaunchKernelGGL(nwc::k_header_digests, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, d.side, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(d.ev_msg, d.side));
    HIP_TRY(hipEventSynchronize(d.ev_cnt[0]));
    if (int rc = leaves(std::min<uint64_t>(nv_host[0], vt), false)) return rc;
    HIP_TRY(hipStreamWaitEvent(s, d.ev_msg, 0));
  }
  hipLaunchKernelGGL(nwc::k_finalize_messages, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, a.rec,
                     a.rec_n, a.hmatch, sbits, lbits, (uint64_t)m, dcodes);
  HIP_TRY(hipGetLastError());
  mark("final queued");
  if (timing && nch > 1) {
    std::string line;
    for (const auto& mk : marks) line += std::string(" ") + mk.first + "@" + std::to_string(mk.second).substr(0, 5);
    std::fprintf(stderr, "nwc sanitize steps:%s\n", line.c_str());
  }
  return 0;
}

static int sanitize_range(int di, const uint8_t* data, const uint64_t* offsets, size_t m, uint64_t gc_round,
                          const uint8_t* vote_target, int32_t* codes, uint8_t* digests32, uint8_t* kinds);

int nwc_sanitize_messages(const uint8_t* data, const uint64_t* offsets, size_t m, uint64_t gc_round,
                          const uint8_t* vote_target, int32_t* codes, uint8_t* digests32, uint8_t* kinds) {
  if (int rc = require_init()) return rc;
  if (m == 0) return 0;
  if (!data || !offsets || !codes) return set_err(NWC_ERR_ARG, "null buffer");
  for (size_t i = 0; i < m; ++i)
    if (offsets[i + 1] < offsets[i]) return set_err(NWC_ERR_ARG, "offsets not monotone at %zu", i);
  // messages are independent: contiguous ranges per device, one host thread each
  return shard(m, [&](int di, uint64_t lo, uint64_t hi) -> int {
    return sanitize_range(di, data, offsets + lo, hi - lo, gc_round, vote_target, codes + lo,
                          digests32 ? digests32 + 32 * lo : nullptr, kinds ? kinds + lo : nullptr);
  });
}

static int sanitize_range(int di, const uint8_t* data, const uint64_t* offsets, size_t m, uint64_t gc_round,
                          const uint8_t* vote_target, int32_t* codes, uint8_t* digests32, uint8_t* kinds) {
  if (m == 0) return 0;
  const uint64_t base = offsets[0], total = offsets[m] - base;
  DevCtx& d = *ctx(di);
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.hip_id));
  if (int rc = ensure_verify_tables(d)) return rc;
  if (!d.cc_stakes) return set_err(NWC_ERR_NOT_INIT, "nwc_set_committee_config has not been called");
  // staging area (the arena): message bytes, offsets, codes, records, digests
  const size_t need = align256(total + 16) + align256(8 * (m + 1)) + align256(4 * m) + align256(16 * m) +
                      align256(32 * m);
  if (int rc = d.ensure_arena(need)) return rc;
  Carve c(d.arena);
  uint8_t* ddata = c.take<uint8_t>(total + 16);
  uint64_t* doff = c.take<uint64_t>(8 * (m + 1));
  int32_t* dcodes = c.take<int32_t>(4 * m);
  uint32_t* drec = c.take<uint32_t>(16 * m);
  uint8_t* ddig = digests32 ? c.take<uint8_t>(32 * m) : nullptr;
  std::vector<uint64_t> hoff(m + 1);
  for (size_t i = 0; i <= m; ++i) hoff[i] = offsets[i] - base;
  const bool staged = total >= ((size_t)4 << 20);
  // Large batches (config 3 from the wire: 10 KB per certificate) go through the pinned stages on
  // the transfer stream in chunks of ~NWC_MSG_CHUNK bytes cut on message boundaries; chunk k is
  // parsed and verified while chunk k + 1 crosses PCIe.  The chunks share the message offsets
  // (uploaded first, relative to ddata) and the message arena (sanitize_dev, run per chunk in
  // stream order).
  static const uint64_t msg_chunk = [] {
    const char* e = std::getenv("NWC_MSG_CHUNK");   // 0 = one copy, then one pass (A/B)
    return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)NWC_MSG_CHUNK;
  }();
  // chunk sizes: from 16 MB doubling up to msg_chunk, and never more than half of what remains
  // (>= 8 MB, so the last one is <= 16 MB): the first parse starts after a short copy, and the
  // work left when the last copy lands (that chunk's parse, leaves and strict equations, the
  // codes) is small; each leaf launch costs >= ~0.18 ms whatever its size, so not smaller
  std::vector<size_t> cuts{0};
  const uint64_t lo = std::min<uint64_t>((uint64_t)8 << 20, msg_chunk);
  if (staged && msg_chunk && total >= 4 * lo) {
    uint64_t at = 0, next = std::min<uint64_t>(msg_chunk, 2 * lo);
    while (total - at > 2 * lo) {
      const uint64_t want = std::max(lo, std::min(next, (total - at) / 2));
      // every cut on a multiple of 64 messages: each chunk's strict launch owns its verdict words
      size_t cm = (size_t)(std::lower_bound(hoff.begin(), hoff.end(), at + want) - hoff.begin()) & ~(size_t)63;
      if (cm <= cuts.back()) cm = cuts.back() + 64;
      if (cm >= m) break;
      cuts.push_back(cm);
      at = hoff[cm];
      next = std::min<uint64_t>(msg_chunk, 2 * next);
    }
    // the last cut on a multiple of 64 messages (the strict launches' verdict words)
    while (cuts.size() > 1 && (cuts.back() & 63)) {
      const size_t c = cuts.back() & ~(size_t)63;
      cuts.pop_back();
      if (c > cuts.back()) cuts.push_back(c);
    }
  }
  cuts.push_back(m);
  const size_t nch = cuts.size() - 1;
  HIP_TRY(hipMemsetAsync(ddata + total, 0, 16, d.stream));
  // the offsets through pinned memory when they fit beside the chunk counts (a pageable source
  // makes the copy wait for the host)
  const size_t hoff_at = 64u << 10;
  if (8 * (m + 1) <= NWC_PINNED_STAGE_MAX - hoff_at) {
    if (int rc = d.ensure_pinned(NWC_PINNED_STAGE_MAX)) return rc;
    uint8_t* const ph = static_cast<uint8_t*>(d.pinned) + hoff_at;
    std::memcpy(ph, hoff.data(), 8 * (m + 1));
    HIP_TRY(hipMemcpyAsync(doff, ph, 8 * (m + 1), hipMemcpyHostToDevice, d.stream));
  } else {
    HIP_TRY(hipMemcpyAsync(doff, hoff.data(), 8 * (m + 1), hipMemcpyHostToDevice, d.stream));
  }
  if (!staged) {
    HIP_TRY(hipMemcpyAsync(ddata, data + base, total, hipMemcpyHostToDevice, d.stream));
    if (int rc = sanitize_dev(d, ddata, doff, m, total, {0, m}, gc_round, vote_target, dcodes, ddig, drec, d.stream))
      return rc;
  } else {
    if (int rc = ensure_stager(d)) return rc;
    while (d.ev_chunk.size() < nch) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      d.ev_chunk.push_back(e);
    }
    // the copies wait for every launch that may still read the arena
    HIP_TRY(hipEventRecord(d.ev_fork, d.stream));
    HIP_TRY(hipStreamWaitEvent(d.xfer, d.ev_fork, 0));
    d.stager->reset();
    const auto tm0 = std::chrono::steady_clock::now();
    std::chrono::steady_clock::time_point tm_copied = tm0;
    // a copy thread fills the stages chunk by chunk and records each chunk's event; this thread
    // runs chunk k once its event has been recorded (a wait on an unrecorded event would not wait)
    std::mutex cmu;
    std::condition_variable ccv;
    size_t recorded = 0;
    hipError_t copy_err = hipSuccess;
    std::thread copier([&] {
      hipError_t e = hipSetDevice(d.hip_id);
      for (size_t k = 0; k < nch && e == hipSuccess; ++k) {
        const uint64_t b0 = hoff[cuts[k]], b1 = hoff[cuts[k + 1]];
        e = d.stager->put(ddata + b0, data + base + b0, b1 - b0);
        if (e == hipSuccess) e = d.stager->flush();
        if (e == hipSuccess) e = hipEventRecord(d.ev_chunk[k], d.xfer);
        if (k + 1 == nch) tm_copied = std::chrono::steady_clock::now();
        std::lock_guard<std::mutex> g(cmu);
        if (e == hipSuccess) recorded = k + 1;
        else copy_err = e;
        ccv.notify_all();
      }
    });
    auto chunk_ready = [&](size_t k) -> int {
      {
        std::unique_lock<std::mutex> g(cmu);
        ccv.wait(g, [&] { return recorded > k || copy_err != hipSuccess; });
        if (recorded <= k) return set_err(NWC_ERR_DEVICE, "message copy: %s", hipGetErrorString(copy_err));
      }
      const hipError_t e = hipStreamWaitEvent(d.stream, d.ev_chunk[k], 0);
      if (e != hipSuccess) return set_err(NWC_ERR_DEVICE, "hipStreamWaitEvent: %s", hipGetErrorString(e));
      return 0;
    };
    auto chunk_queued = [&](size_t k) -> bool {
      std::lock_guard<std::mutex> g(cmu);
      return recorded > k;
    };
    int rc = sanitize_dev(d, ddata, doff, m, total, cuts, gc_round, vote_target, dcodes, ddig, drec, d.stream,
                          chunk_ready, chunk_queued);
    copier.join();   // the copier never waits on this thread: it runs through every chunk
    if (rc) {
      (void)hipStreamSynchronize(d.xfer);   // no copy still writes the arena when the call returns
      return rc;
    }
    if (host_timing()) {
      HIP_TRY(hipStreamSynchronize(d.stream));
      const auto tm1 = std::chrono::steady_clock::now();
      std::fprintf(stderr, "nwc sanitize: %zu messages, %.1f MB in %zu chunks: copies queued after %.2f ms, pipeline done %.2f ms later\n",
                   m, total / 1e6, nch, std::chrono::duration<double>(tm_copied - tm0).count() * 1e3,
                   std::chrono::duration<double>(tm1 - tm_copied).count() * 1e3);
    }
  }
  HIP_TRY(hipMemcpyAsync(codes, dcodes, 4 * m, hipMemcpyDeviceToHost, d.stream));
  std::vector<uint32_t> rec;
  if (kinds) {
    rec.resize(4 * m);
    HIP_TRY(hipMemcpyAsync(rec.data(), drec, 16 * m, hipMemcpyDeviceToHost, d.stream));
  }
  if (digests32) HIP_TRY(hipMemcpyAsync(digests32, ddig, 32 * m, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  if (kinds)
    for (size_t i = 0; i < m; ++i) kinds[i] = (uint8_t)rec[4 * i];
  return 0;
}

int nwc_dev_sanitize_messages(const void* d_data, const void* d_offsets, uint64_t m, uint64_t total,
                              uint64_t gc_round, const uint8_t* vote_target, void* d_codes, void* d_digests32,
                              void* stream) {
  if (int rc = require_init()) return rc;
  if (m == 0) return 0;
  if (!d_data || !d_offsets || !d_codes) return set_err(NWC_ERR_ARG, "null buffer");
  if ((reinterpret_cast<uintptr_t>(d_data) & 3) != 0) return set_err(NWC_ERR_ARG, "d_data must be 4-byte aligned");
  DevCtx& d = *ctx(t_dev < (int)g_devs.size() ? t_dev : 0);
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.hip_id));
  if (!d.cc_stakes) return set_err(NWC_ERR_NOT_INIT, "nwc_set_committee_config has not been called");
  return sanitize_dev(d, static_cast<const uint8_t*>(d_data), static_cast<const uint64_t*>(d_offsets), m, total,
                      {0, (size_t)m}, gc_round, vote_target, static_cast<int32_t*>(d_codes), static_cast<uint8_t*>(d_digests32),
                      nullptr, stream ? static_cast<hipStream_t>(stream) : d.stream);
}

}  // extern "C"

#include "digester.h"

extern "C" {

int nwc_memory_info(nwc_memory* out) {
  if (int rc = require_init()) return rc;
  if (!out) return set_err(NWC_ERR_ARG, "null argument");
  DevCtx* dp = ctx(t_dev);
  if (!dp) return set_err(NWC_ERR_ARG, "device index %d not initialised", t_dev);
  DevCtx& d = *dp;
  *out = nwc_memory{};
  {
    std::lock_guard<std::mutex> lk(d.mu);
    // built by the first call that verifies or signs (ensure_verify_tables); 0 before
    out->tables = !d.tables_ready ? 0 :
                  2 * 129 * sizeof(nwc::ge_niels) + 2 * (size_t)nwc::B24_ENTRIES * sizeof(nwc::ge_niels_pad) +
                  2 * sizeof(nwc::ge_p3) + nwc::BaseComb::per * sizeof(nwc::ge_niels_pad) +
                  (d.comb16 ? nwc::COMB16_TOTAL * sizeof(nwc::ge_niels_pad) + nwc::COMB16_WINDOWS * sizeof(nwc::ge_p3) : 0) +
                  36 * (size_t)NWC_MEMO_SLOTS;
    out->committee = d.cm_bytes;
    out->auto_cache = (size_t)d.ak_cap * (36 + 129 * sizeof(nwc::ge_niels) + nwc::COMB_PER_KEY * sizeof(nwc::ge_niels_pad)) +
                      4 * (size_t)d.ak_slot_cap + d.kb_cap * sizeof(nwc::ge_p3) +
                      (d.lk_alloc ? (size_t)nwc::LK_MAX_KEYS * (36 + nwc::KeyComb::windows * sizeof(nwc::ge_p3)) +
                                        (size_t)d.lk.cap * nwc::COMB_PER_KEY * sizeof(nwc::ge_niels_pad) +
                                        4 * (size_t)nwc::LK_SLOTS + 16
                                  : 0);
    out->scratch = d.scratch_cap + d.straus_cap + d.msm_cap + d.rs_cap + d.arena_cap + d.msg_arena_cap + 12 * d.fb_cap + d.pair_cap + d.sign_cap +
                   8 * (size_t)d.ts_slot_count;
  }
  out->digesters = digester_device_bytes(d.hip_id);
  size_t fr = 0, tot = 0;
  HIP_TRY(hipSetDevice(d.hip_id));
  HIP_TRY(hipMemGetInfo(&fr, &tot));
  out->device_free = fr;
  out->device_total = tot;
  return 0;
}

int nwc_trim(void) {
  if (int rc = require_init()) return rc;
  DevCtx* dp = ctx(t_dev);
  if (!dp) return set_err(NWC_ERR_ARG, "device index %d not initialised", t_dev);
  DevCtx& d = *dp;
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.hip_id));
  // every stream: nwc_dev_* launches on callers' streams read these buffers too
  HIP_TRY(hipDeviceSynchronize());
  if (d.scratch) HIP_TRY(hipFree(d.scratch));
  if (d.straus_scratch) HIP_TRY(hipFree(d.straus_scratch));
  if (d.msm_scratch) HIP_TRY(hipFree(d.msm_scratch));
  d.msm_scratch = nullptr; d.msm_cap = 0;
  if (d.rs_buf) HIP_TRY(hipFree(d.rs_buf));
  d.rs_buf = nullptr; d.rs_cap = 0;
  if (d.pair_buf) HIP_TRY(hipFree(d.pair_buf));
  d.pair_buf = nullptr; d.pair_cap = 0;
  if (d.sign_buf) HIP_TRY(hipFree(d.sign_buf));
  d.sign_buf = nullptr; d.sign_cap = 0;
  if (d.arena) HIP_TRY(hipFree(d.arena));
  if (d.msg_arena) HIP_TRY(hipFree(d.msg_arena));
  d.scratch = nullptr; d.scratch_cap = 0;
  d.straus_scratch = nullptr; d.straus_cap = 0;
  d.arena = nullptr; d.arena_cap = 0;
  d.msg_arena = nullptr; d.msg_arena_cap = 0;
  // the per-launch lists (fallback, uncached, torsion hash set) and the launch-key set (2.6 GB of
  // combs): the next launch that needs them allocates them again, the launch keys empty
  free_lists(d);
  if (d.lk_alloc) {
    for (void* p : {(void*)d.lk.keys, (void*)d.lk.flags, (void*)d.lk.slots, (void*)d.lk.comb, (void*)d.lk.bases,
                    (void*)d.lk.state})
      HIP_TRY(hipFree(p));
    d.lk = nwc::LaunchKeys{};
    d.lk_alloc = false;
  }
  return 0;
}

}  // extern "C"
