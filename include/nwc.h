/*
 * nwc.h -- C ABI of the MI355X-native Narwhal signature-and-digest hot path (libnwc.so).
 *
 * This is the drop-in boundary: the reference's `crypto` crate keeps its Rust API and calls
 * these entry points through a thin FFI shim.  Every entry point names the
 * reference interface it replaces (paths under /root/reference).
 *
 * Conventions
 *   - Plain pointers and sizes only; all buffers are caller-owned.  Host entry points take
 *     host memory; `nwc_dev_*` entry points take device (HBM) pointers and a hipStream_t
 *     passed as void* (NULL = the library's own stream) and are asynchronous on it.
 *   - Single verdicts: 0 = valid (Rust `Ok(())`), 1 = invalid (`Err(CryptoError)`),
 *     < 0 = runtime/device/argument error (never reported as "invalid"; the Rust shim panics).
 *   - Batch calls return 0 on success (< 0 on error) and fill bitmaps: bit i of a bitmap is
 *     byte i/8, bit i%8 (LSB first); 1 = valid for verdict bitmaps, 1 = bad for bad-vote bitmaps.
 *     Device bitmaps are arrays of uint64_t words with the same bit order.
 *   - Messages at the crypto surface are always 32-byte `Digest`s (crypto/src/lib.rs:203,214).
 *   - Thread-safe and reentrant (tokio tasks call concurrently: worker/src/worker.rs:182,227).
 */
#ifndef NWC_H
#define NWC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NWC_OK 0
#define NWC_INVALID 1
#define NWC_ERR_DEVICE (-1)
#define NWC_ERR_ARG (-2)
#define NWC_ERR_NOT_INIT (-3)
#define NWC_ERR_NO_DEVICE (-4)

/* ---- lifecycle ------------------------------------------------------------------------ */
/* Node start-up hook (node/src/main.rs:69-134).  device_mask: bit d = use HIP device d
 * (0 = device 0).  Builds the basepoint table on each device.  Idempotent. */
int nwc_init(uint32_t device_mask);
void nwc_shutdown(void);
/* Text of the last error on the calling thread ("" if none). */
const char* nwc_last_error(void);
/* ABI version (major << 16 | minor). */
int nwc_version(void);
/* Number of devices initialised. */
int nwc_device_count(void);
/* Identity of this build: a hash over the library's sources (narwhal_amd/csrc, this header)
 * and compile flags, computed by narwhal_amd/build.py, so a caller or test can check that the
 * binary it loaded was compiled from the tree it came with.  "unknown" for other builds. */
const char* nwc_build_id(void);

/* ---- device memory (a primary and a worker may share one GPU) ------------------------ */
/* Bytes held by this process on the calling thread's device (nwc_dev_set_device): tables =
 * basepoint tables (radix-2^24 ladder tables 2.1 GB, radix-2^22 comb 3.2 GB unless NWC_COMB16=0,
 * small ones), built by the first call that verifies or signs -- 0 in a process that only digests;
 * committee = the nwc_set_committee cache (20 MB per key with combs); auto_cache = the auto key
 * cache (NWC_AUTO_KEYS) and the launch keys (20 MB of comb per key that joined); scratch =
 * per-launch buffers grown on demand (ladder tables, Straus tables, MSM groups, staging, message
 * buffers; the batch entries' buffers above NWC_VERIFY_KEEP_BYTES are freed by the next launch of
 * another path); digesters = the device buffers of live nwc_digesters on this device;
 * device_free / device_total = hipMemGetInfo. */
typedef struct nwc_memory {
  uint64_t tables, committee, auto_cache, scratch, digesters, device_free, device_total;
} nwc_memory;
int nwc_memory_info(nwc_memory* out);
/* Frees the calling thread's device's on-demand scratch (re-allocated by the next call that
 * needs it); waits for the device to be idle.  Tables and caches stay. */
int nwc_trim(void);

/* Test / A-B knobs, settable at run time instead of through the environment (which is read
 * once): "straus_nq" = votes per sub-batch of nwc_dev_verify_batch_straus (1..16, default 12,
 * env NWC_STRAUS_NQ); "force_windows" = half-ladder windows forced on every wave (33..37, 0 = off,
 * env NWC_FORCE_WINDOWS; verdicts must not change); "launch_keys" = 0 / 1 (default 1, env
 * NWC_LAUNCH_KEYS; nwc_launch_keys_info); "msm_group" = votes per Pippenger group of the MSM
 * entry (a multiple of 64 in 64..4096; 0, the default = sized per launch; env NWC_MSM_GROUP);
 * "msm_adapt" = 0 / 1 (default 1, env NWC_MSM_ADAPT): the MSM entry's skip policy (0 = the
 * equation on every group); "dalek_seed" = a fixed 32-bit seed of the batch entries' random z_i
 * (z_i = SHA-512(seed as 4 LE bytes || 28 zero bytes || u64le(i))[..16]; 0, the default = 32 bytes
 * of the host CSPRNG per launch), so tests can compute dalek's equation for the same z_i.
 * NWC_ERR_ARG for an unknown name or value.
 * Not part of the crate's API. */
int nwc_diag_set(const char* name, int64_t value);

/* The shader clock the headline kernel holds under load: one launch of a diagnostic build of the
 * strict verification kernel (k_verify with in-kernel stamps; the verdict path never runs it) on
 * the caller's device inputs, as nwc_dev_verify(.., strict = 1, ..), synchronised on `stream`.
 * Every wave stamps s_memtime / s_memrealtime at entry and exit; *clock_ghz = the median over
 * waves of delta(memtime) / delta(realtime) x 100 MHz, *waves = the waves counted.  Call it after
 * some seconds of back-to-back launches (MI355X_MICROARCH.md, DVFS item 6).  The verdict words
 * are written as by nwc_dev_verify.  NWC_ERR_ARG with a committee cache set (strict launches would
 * take the comb kernel, which has no stamps) or n > NWC_VERIFY_MAX_LAUNCH (a split launch).
 * Diagnostics only, not part of the crate's API. */
int nwc_diag_verify_clock(const void* d_msgs, uint64_t msg_stride, const void* d_pks, const void* d_sigs, uint64_t n,
                          void* d_verdict_words, void* stream, double* clock_ghz, uint32_t* waves);

/* ---- verification ----------------------------------------------------------------------- */
/* crypto::Signature::verify -> dalek verify_strict.  Replaces crypto/src/lib.rs:200-204
 * (called from primary/src/messages.rs:63-66 Header::verify and :138-141 Vote::verify). */
int nwc_verify_strict(const uint8_t msg32[32], const uint8_t pk[32], const uint8_t sig[64]);

/* crypto::Signature::verify_batch(digest, votes).  Replaces crypto/src/lib.rs:206-219
 * (called from primary/src/messages.rs:214 Certificate::verify).  Votes are n (pk, sig) pairs
 * laid out as pks[32*n], sigs[64*n].  n == 0 -> valid.  bad_bitmap (nullable, ceil(n/8)
 * bytes) receives the exact set of failing votes (the per-signature leaf). */
int nwc_verify_batch(const uint8_t msg32[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                     uint8_t* bad_bitmap);

/* n independent Signature::verify calls (BASELINE configs 2 and 5). */
int nwc_verify_strict_many(const uint8_t* msgs32, const uint8_t* pks, const uint8_t* sigs, size_t n,
                           uint8_t* verdict_bitmap);

/* m certificates (BASELINE config 3): certificate c has digest digests[32c] and votes
 * [offsets[c], offsets[c+1]) of pks/sigs; offsets[0] must be 0.  cert_ok_bitmap: m bits,
 * bad_vote_bitmap (nullable): offsets[m] bits. */
int nwc_verify_batch_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks,
                          const uint8_t* sigs, size_t m, uint8_t* cert_ok_bitmap,
                          uint8_t* bad_vote_bitmap);
/* The same m certificates through dalek's own batch equation (ed25519-dalek 1.0.1 batch.rs, the
 * algorithm behind crypto/src/lib.rs:218): random 128-bit z_i, one Straus pass per sub-batch of
 * ~12 votes on the GPU (nwc_dev_verify_batch_straus), the exact per-vote leaves for the sub-batches
 * it rejects.  Same verdicts and bad sets as nwc_verify_batch_many on the deterministic domain; on
 * dalek's randomized domain (pure-torsion residuals, torsion-bearing keys) dalek's probabilities
 * instead of Err.  Faster on clean traffic, slower at ~1 % bad votes. */
int nwc_verify_batch_straus_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks,
                                 const uint8_t* sigs, size_t m, uint8_t* cert_ok_bitmap,
                                 uint8_t* bad_vote_bitmap);

/* The same m certificates with dalek's batch semantics (crypto/src/lib.rs:218):
 * each certificate passes iff dalek's equation holds for it with random 128-bit z_i.  Where key
 * combs apply (a committee cache, or >= 65,536 votes whose keys repeat: launch keys) every vote is
 * first decided by the exact leaf on the comb path; then dalek's equation is evaluated once per
 * certificate over the votes the leaves rejected (the others contribute the identity whatever
 * z_i is), exactly, in the 8-torsion group -- the deterministic domain is the leaves' verdict, and
 * on the randomized one (pure-torsion residuals, torsion-bearing keys) a certificate passes with
 * dalek's probability, its failing votes then cleared from the bad set.  Otherwise the Pippenger
 * MSM per group of up to 4,096 consecutive votes (nwc_dev_verify_batch_msm) decides first and the
 * votes of the groups it rejects go to the exact leaves.  Every vote meets at most one random
 * equation: its certificate's, or (no combs) its group's. */
int nwc_verify_batch_msm_many(const uint8_t* digests, const uint32_t* offsets, const uint8_t* pks,
                              const uint8_t* sigs, size_t m, uint8_t* cert_ok_bitmap,
                              uint8_t* bad_vote_bitmap);

/* Committee key cache (config/src/lib.rs:154-156 Committee).  Optional: verdicts never
 * depend on it. */
int nwc_set_committee(const uint8_t* pks, size_t n);

/* Key caches of the calling thread's device (nwc_dev_set_device): keys in the committee cache,
 * and in the auto key cache -- keys of small host calls (<= 1024 equations) outside the
 * committee cache, added the second time they are seen, so that a node's repeated certificates
 * take the latency kernel without nwc_set_committee (NWC_AUTO_KEYS = capacity, 0 = off).
 * Diagnostics only: verdicts never depend on either cache.  Not part of the crate's API. */
int nwc_cache_stats(uint32_t* committee_keys, uint32_t* auto_keys);

/* Auto key cache lifecycle of the calling thread's device: capacity (NWC_AUTO_KEYS), insert
 * batches built so far, and calls served by the latency kernel over it.  Once full, new keys
 * replace the oldest (FIFO); nwc_set_committee empties it.  Any pointer may be NULL.
 * Diagnostics only, not part of the crate's API. */
int nwc_auto_cache_info(uint32_t* capacity, uint64_t* builds, uint64_t* hits);

/* Launch keys of the calling thread's device: a batch-leaf launch of >= 65,536 equations without a
 * committee cache samples its keys, and keys it repeats (>= ~1/4096 of the sample) join a
 * device-resident set with their flags and radix-2^14 combs (built once; room for 20 MB of comb
 * per key is reserved as keys ask to join: the first launch measures its demand, later ones grow
 * it from the demand the previous launch recorded, so a key that did not fit joins at the next
 * launch), so that votes of a committee the caller never registered take the comb kernel --
 * cross-certificate key aggregation, no nwc_set_committee needed.  Up to `capacity` keys; emptied by nwc_set_committee
 * and nwc_trim, and replaced by a launch whose repeated keys do not fit while the held ones cover
 * less than a quarter of its sample (a new committee); NWC_LAUNCH_KEYS=0 (or
 * nwc_diag_set("launch_keys", 0)) turns it off.
 * Verdicts never depend on it.  Waits for the device.  Diagnostics only. */
int nwc_launch_keys_info(uint32_t* held, uint32_t* capacity);

/* ---- worker batch digests behind a Processor-shaped queue (worker/src/processor.rs:35-55) ----
 * Replaces the Processor's per-batch `Sha512::digest(&batch)[..32]` (:38) for workers that can
 * hand batches over in groups.  A digester owns a drain thread on the calling thread's device
 * (nwc_dev_set_device): it takes the first submitted batch, then whatever else arrives within
 * max_wait_us (up to max_group batches), and digests the group with one GPU launch on its own
 * stream.  Batches are BORROWED: the caller keeps each one alive until its digest has been
 * polled (the Processor stores the batch after hashing it anyway).  Digests come back in
 * submission order with the caller's tag.  One 500-KB batch alone takes ~28 ms on the GPU (a
 * sequential SHA-512 chain on one lane) against ~0.36 ms on one host core: measured, the GPU ties 16
 * host cores at ~1,000 batches per group and is ~3.8x faster at 100,000 (PCIe-bound, ~40 GB/s;
 * 54 GB/s from the receive arena below).  Data path: NWC_DIGEST_STAGES (4) pinned 32-MB stages filled by
 * NWC_DIGEST_COPY_THREADS (8) host threads; one launch holds at most NWC_DIGEST_MAX_BYTES
 * (16 GiB) of batches in HBM (larger groups are cut), and a device buffer above
 * NWC_DIGEST_KEEP_BYTES (1 GiB) is freed after its group.  create returns NULL on failure
 * (nwc_last_error).  poll waits up to wait_us for a result and returns one run of results with
 * the same status: digests (returns 0), or the tags of a group that failed on the device (returns
 * the error code < 0; digests32 zeroed) -- every submitted tag comes back exactly once, in order.
 * After a failure submit refuses new batches, and poll returns the error (n_done = 0) once every
 * batch submitted before it has come back.  destroy digests what is queued, wakes threads blocked in poll and
 * waits for them to leave, then frees the digester (no call on it may start after destroy). */
typedef struct nwc_digester nwc_digester;
nwc_digester* nwc_digester_create(uint32_t max_group, uint32_t max_wait_us);
int nwc_digester_submit(nwc_digester* q, const uint8_t* batch, size_t len, uint64_t tag);
int nwc_digester_poll(nwc_digester* q, size_t max, uint32_t wait_us, uint64_t* tags, uint8_t* digests32,
                      size_t* n_done);
int nwc_digester_stats(nwc_digester* q, uint64_t* groups, uint64_t* batches, uint64_t* bytes);
/* Receive arena: `bytes` of pinned host memory owned by the digester (freed by destroy), for a
 * worker that receives batches straight into it (the network read's destination, instead of a
 * Vec the Processor later hands over).  A group whose batches all lie in the arena, each placed
 * at the previous one's offset + its length rounded up to 16 bytes (starts 16-byte aligned),
 * skips the stage fill: each contiguous run of batches is one DMA from the arena into HBM (at most
 * 1,024 runs per group; otherwise, or with any batch outside the arena, the group takes the stage
 * path).  Batches stay borrowed as with any submit: do not overwrite a batch's bytes before its
 * digest has been polled.  Create it before the first submit; a later call returns the same
 * arena if `bytes` fits.  Returns NULL on failure (nwc_last_error).  No counterpart in the
 * reference (its Processor gets a Vec<u8>). */
uint8_t* nwc_digester_arena(nwc_digester* q, size_t bytes);
/* Groups that took the arena's direct path so far (diagnostics). */
int nwc_digester_direct_groups(nwc_digester* q, uint64_t* direct_groups);
int nwc_digester_destroy(nwc_digester* q);

/* ---- primary messages ---------------------------------------- */
/* config::Committee for the message checks (config/src/lib.rs:134-212): n authorities with
 * their keys, stakes (Committee::stake) and worker ids (Committee::worker): authority k runs
 * workers worker_ids[worker_offsets[k] .. worker_offsets[k+1]).  Also sets the key cache
 * (nwc_set_committee); a later nwc_set_committee drops the stake/worker tables.  At most 4096
 * authorities. */
int nwc_set_committee_config(const uint8_t* pks, const uint64_t* stakes, size_t n,
                             const uint32_t* worker_offsets, const uint32_t* worker_ids);

/* DagError codes of nwc_sanitize_messages (primary/src/error.rs) */
#define NWC_DAG_OK 0
#define NWC_DAG_INVALID_SIGNATURE 1
#define NWC_DAG_INVALID_HEADER_ID 2
#define NWC_DAG_MALFORMED_HEADER 3
#define NWC_DAG_UNKNOWN_AUTHORITY 4
#define NWC_DAG_AUTHORITY_REUSE 5
#define NWC_DAG_CERTIFICATE_REQUIRES_QUORUM 6
#define NWC_DAG_TOO_OLD 7
#define NWC_DAG_SERIALIZATION_ERROR 8
#define NWC_DAG_UNEXPECTED_VOTE 9
#define NWC_DAG_UNEXPECTED_MESSAGE 10
/* not a DagError: decoding a PublicKey whose base64 gives < 32 bytes panics in the reference
 * (crypto/src/lib.rs:75 `bytes[..32]`, inside bincode::deserialize at primary/src/primary.rs:230) */
#define NWC_DAG_DECODE_PANIC 11

/* Core::sanitize_header / sanitize_vote / sanitize_certificate (primary/src/core.rs:306-346)
 * for a batch of wire messages, each the bincode bytes of a PrimaryMessage as received by
 * PrimaryReceiverHandler::dispatch (primary/src/primary.rs:224-240): message i is
 * data[offsets[i] .. offsets[i+1]).  Decoding (incl. the base64 PublicKeys), Header::digest,
 * Vote::digest, Certificate::digest, the committee checks of Header::verify / Vote::verify /
 * Certificate::verify (primary/src/messages.rs:48-67, 131-142, 189-215) and every signature run
 * on the GPU.  gc_round: TooOld for headers and certificates (0 disables).  vote_target
 * (nullable, 72 B = id || round u64 LE || origin): the current header of sanitize_vote.
 * codes[i] = NWC_DAG_*; digests32 (nullable): the message's digest; kinds (nullable):
 * 0 header, 1 vote, 2 certificate, 3 other.  Needs nwc_set_committee_config. */
int nwc_sanitize_messages(const uint8_t* data, const uint64_t* offsets, size_t m, uint64_t gc_round,
                          const uint8_t* vote_target, int32_t* codes, uint8_t* digests32, uint8_t* kinds);

/* Device-resident variant: d_data (4-byte aligned, >= 16 readable bytes past the last message)
 * and d_offsets (device u64[m+1], d_offsets[0] = 0, d_offsets[m] = total) in HBM; d_codes device
 * i32[m], d_digests32 (nullable) device m x 32 B.  Synchronises once (the vote count). */
int nwc_dev_sanitize_messages(const void* d_data, const void* d_offsets, uint64_t m, uint64_t total,
                              uint64_t gc_round, const uint8_t* vote_target, void* d_codes,
                              void* d_digests32, void* stream);

/* ---- digests -------------------------------------------------------------------------- */
/* Sha512::digest(bytes)[..32] -- worker/src/processor.rs:38 and crypto's `Hash for &[u8]`
 * (crypto/src/tests/crypto_tests.rs:8-12). */
int nwc_digest32(const uint8_t* data, size_t len, uint8_t out32[32]);
/* n messages data[offsets[i] .. offsets[i+1]) -> out32[32*i]. */
int nwc_sha512_trunc32_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32);

/* ---- device-resident variants (inputs already in HBM) ---------------------------------- */
/* strict != 0: verify_strict semantics; strict == 0: batch-leaf semantics.  msg_index
 * (nullable, device u32[n]) selects the digest of equation i; otherwise digest i*msg_stride.
 * n < 2^32 per call (NWC_ERR_ARG otherwise). */
int nwc_dev_verify(const void* d_msgs, const void* d_msg_index, uint64_t msg_stride,
                   const void* d_pks, const void* d_sigs, uint64_t n, int strict,
                   void* d_verdict_words, void* stream);
/* Per-certificate AND of leaf verdict words (d_offsets: device u32[m+1]). */
int nwc_dev_cert_reduce(const void* d_leaf_words, const void* d_offsets, uint64_t m, uint64_t nvotes,
                        void* d_cert_words, void* d_bad_words, void* stream);
/* Signature::verify_batch over m certificates as dalek's own batch equation (crypto/src/lib.rs:
 * 206-219; ed25519-dalek 1.0.1 batch.rs) over sub-batches of ~12 consecutive votes (any
 * certificates; NWC_STRAUS_NQ overrides): sum z_i R_i + sum (z_i k_i mod l) A_i -
 * (sum z_i s_i mod l) B == O with random 128-bit z_i, one Straus pass with shared doublings per
 * lane (k_verify_straus); the votes of sub-batches it rejects are then re-decided by the exact
 * per-vote leaves, so d_leaf_words (a bit per vote, as nwc_dev_verify's) feeds nwc_dev_cert_reduce
 * for the certificate verdicts and the exact bad-vote set.  d_offsets: m + 1 uint32 vote offsets
 * (checked non-null; the sub-batches do not follow them); d_msg_index: the certificate of each
 * vote.  Same verdicts and bad sets as the leaf path on the deterministic domain; on dalek's
 * randomized domain (pure-torsion residuals, torsion-bearing keys) a vote's sub-batch passes with
 * dalek's probability (~1/ord) where the leaf path answers Err.  Without the basepoint comb
 * (NWC_COMB16=0) it runs the leaves. */
int nwc_dev_verify_batch_straus(const void* d_digests, const void* d_offsets, const void* d_msg_index, uint64_t m,
                                uint64_t nvotes, const void* d_pks, const void* d_sigs, void* d_leaf_words,
                                void* stream);
/* Signature::verify_batch over m certificates with dalek's batch semantics, device-resident (as
 * nwc_verify_batch_msm_many).  With key combs (committee cache, or launch keys at >= 65,536 votes):
 * the comb-path leaves, then dalek's equation per certificate over the leaves' failing votes, in
 * E[8].  Without: dalek's batch equation as a Pippenger MSM per group of
 * consecutive votes (up to 4,096, sized so the groups fill whole rounds of the resident waves;
 * NWC_MSM_GROUP / nwc_diag_set("msm_group") fixes it): one wave per group sorts its points into 512
 * buckets per 10-bit window in LDS and reduces the buckets across its 64 lanes; the votes of groups
 * that fail go to the exact per-vote leaves (no second random equation: on dalek's randomized
 * domain a vote passes iff its group's equation holds).  Skip policy (device-side, no host
 * synchronisation; its state is per device, shared by every caller and stream of the device): when
 * more than half of a launch's groups fail (a bad-vote rate of about one per group or more), the next
 * 7 launches skip the equation and hand every vote straight to the leaves; the one after them runs
 * it on every group again and decides anew.  d_leaf_words as nwc_dev_verify_batch_straus's. */
int nwc_dev_verify_batch_msm(const void* d_digests, const void* d_offsets, const void* d_msg_index, uint64_t m,
                             uint64_t nvotes, const void* d_pks, const void* d_sigs, void* d_leaf_words,
                             void* stream);
/* Groups of the MSM entry on the calling thread's device since nwc_init: passed (their votes'
 * bits set by the equation), failed (re-decided by the leaves), of the failed ones, groups with
 * more distinct keys than the LDS key table holds (126), and groups the skip policy handed to the
 * leaves without the equation.  Any pointer may be null.  Waits for the device.  Diagnostics
 * only. */
int nwc_msm_stats(uint64_t* groups_passed, uint64_t* groups_failed, uint64_t* key_overflows, uint64_t* groups_skipped);
int nwc_dev_sha512_trunc32(const void* d_data, const void* d_offsets, uint64_t n, void* d_out32,
                           void* stream);
/* Same, message i = d_data[d_starts[i] .. d_ends[i]) (device u64 arrays): any layout, e.g. a
 * pool of resident batches hashed repeatedly.  Starts 16-byte aligned take the fast path. */
int nwc_dev_sha512_trunc32_ranges(const void* d_data, const void* d_starts, const void* d_ends, uint64_t n,
                                  void* d_out32, void* stream);
/* Synthetic workload generation (BASELINE configs 2/3/5): out_i = SHA-512(tag||u64le(first+i))[..32]
 * and RFC 8032 keygen+sign of (seed_i, msg_i). */
int nwc_dev_derive32(const uint8_t* tag, int taglen, uint64_t first, uint64_t n, void* d_out,
                     void* stream);
int nwc_dev_keygen_sign(const void* d_seeds, const void* d_msgs, uint64_t n, void* d_pks,
                        void* d_sigs, void* stream);
/* Select the HIP device used by nwc_dev_* on the calling thread (index into the init mask). */
int nwc_dev_set_device(int device);

/* ---- sharding (host only; no device needed) --------------------------------------------- */
/* independent units split over `world` GPUs/ranks.  [*lo, *hi) of n units for
 * `rank`: contiguous, every shard but the last starts on a multiple of 64 (whole verdict words),
 * so shards never share a byte of a verdict bitmap.  Used by the host entry points' per-device
 * threads and mirrored by narwhal_amd/shard.py shard_bounds for one-process-per-GPU runs. */
int nwc_shard_bounds(uint64_t n, uint32_t world, uint32_t rank, uint64_t* lo, uint64_t* hi);
/* Vote-index cuts (world + 1 values, cuts[0] = 0, cuts[world] = offsets[m]) on certificate
 * boundaries, balanced by vote count: a certificate's votes never split (config 3). */
int nwc_cert_cuts(const uint32_t* offsets, size_t m, uint32_t world, uint64_t* cuts);

#ifdef __cplusplus
}
#endif
#endif /* NWC_H */
