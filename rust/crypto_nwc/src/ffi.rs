//! Raw declarations of every entry point of include/nwc.h (checked against the header by
//! tests/test_rust_shim.py: same names, same parameter types, same order).
#![allow(dead_code)]
use std::os::raw::{c_char, c_int, c_void};

/// Opaque handle of a batch digester (nwc_digester_create).
#[allow(non_camel_case_types)]
pub enum nwc_digester {}

/// Device bytes this process holds on one device (nwc_memory_info).
#[allow(non_camel_case_types)]
#[repr(C)]
#[derive(Default, Debug, Clone, Copy)]
pub struct nwc_memory {
    pub tables: u64,
    pub committee: u64,
    pub auto_cache: u64,
    pub scratch: u64,
    pub digesters: u64,
    pub device_free: u64,
    pub device_total: u64,
}

#[link(name = "nwc")]
extern "C" {
    pub fn nwc_init(device_mask: u32) -> c_int;
    pub fn nwc_shutdown();
    pub fn nwc_last_error() -> *const c_char;
    pub fn nwc_version() -> c_int;
    pub fn nwc_device_count() -> c_int;
    pub fn nwc_build_id() -> *const c_char;
    pub fn nwc_memory_info(out: *mut nwc_memory) -> c_int;
    pub fn nwc_trim() -> c_int;
    pub fn nwc_diag_set(name: *const c_char, value: i64) -> c_int;
    pub fn nwc_diag_verify_clock(d_msgs: *const c_void, msg_stride: u64, d_pks: *const c_void, d_sigs: *const c_void,
                                 n: u64, d_verdict_words: *mut c_void, stream: *mut c_void, clock_ghz: *mut f64,
                                 waves: *mut u32) -> c_int;

    pub fn nwc_verify_strict(msg32: *const u8, pk: *const u8, sig: *const u8) -> c_int;
    pub fn nwc_verify_batch(msg32: *const u8, pks: *const u8, sigs: *const u8, n: usize, bad_bitmap: *mut u8) -> c_int;
    pub fn nwc_verify_strict_many(msgs32: *const u8, pks: *const u8, sigs: *const u8, n: usize,
                                  verdict_bitmap: *mut u8) -> c_int;
    pub fn nwc_verify_batch_many(digests: *const u8, offsets: *const u32, pks: *const u8, sigs: *const u8, m: usize,
                                 cert_ok_bitmap: *mut u8, bad_vote_bitmap: *mut u8) -> c_int;
    pub fn nwc_verify_batch_straus_many(digests: *const u8, offsets: *const u32, pks: *const u8, sigs: *const u8,
                                        m: usize, cert_ok_bitmap: *mut u8, bad_vote_bitmap: *mut u8) -> c_int;
    pub fn nwc_verify_batch_msm_many(digests: *const u8, offsets: *const u32, pks: *const u8, sigs: *const u8,
                                        m: usize, cert_ok_bitmap: *mut u8, bad_vote_bitmap: *mut u8) -> c_int;
    pub fn nwc_set_committee(pks: *const u8, n: usize) -> c_int;
    pub fn nwc_cache_stats(committee_keys: *mut u32, auto_keys: *mut u32) -> c_int;
    pub fn nwc_auto_cache_info(capacity: *mut u32, builds: *mut u64, hits: *mut u64) -> c_int;
    pub fn nwc_launch_keys_info(held: *mut u32, capacity: *mut u32) -> c_int;

    pub fn nwc_set_committee_config(pks: *const u8, stakes: *const u64, n: usize, worker_offsets: *const u32,
                                    worker_ids: *const u32) -> c_int;
    pub fn nwc_sanitize_messages(data: *const u8, offsets: *const u64, m: usize, gc_round: u64, vote_target: *const u8,
                                 codes: *mut i32, digests32: *mut u8, kinds: *mut u8) -> c_int;
    pub fn nwc_dev_sanitize_messages(d_data: *const c_void, d_offsets: *const c_void, m: u64, total: u64, gc_round: u64,
                                     vote_target: *const u8, d_codes: *mut c_void, d_digests32: *mut c_void,
                                     stream: *mut c_void) -> c_int;

    pub fn nwc_digest32(data: *const u8, len: usize, out32: *mut u8) -> c_int;
    pub fn nwc_sha512_trunc32_many(data: *const u8, offsets: *const u64, n: usize, out32: *mut u8) -> c_int;
    pub fn nwc_digester_create(max_group: u32, max_wait_us: u32) -> *mut nwc_digester;
    pub fn nwc_digester_submit(q: *mut nwc_digester, batch: *const u8, len: usize, tag: u64) -> c_int;
    pub fn nwc_digester_poll(q: *mut nwc_digester, max: usize, wait_us: u32, tags: *mut u64, digests32: *mut u8,
                             n_done: *mut usize) -> c_int;
    pub fn nwc_digester_stats(q: *mut nwc_digester, groups: *mut u64, batches: *mut u64, bytes: *mut u64) -> c_int;
    pub fn nwc_digester_destroy(q: *mut nwc_digester) -> c_int;
    pub fn nwc_digester_arena(q: *mut nwc_digester, bytes: usize) -> *mut u8;
    pub fn nwc_digester_direct_groups(q: *mut nwc_digester, direct_groups: *mut u64) -> c_int;

    pub fn nwc_dev_verify(d_msgs: *const c_void, d_msg_index: *const c_void, msg_stride: u64, d_pks: *const c_void,
                          d_sigs: *const c_void, n: u64, strict: c_int, d_verdict_words: *mut c_void,
                          stream: *mut c_void) -> c_int;
    pub fn nwc_dev_cert_reduce(d_leaf_words: *const c_void, d_offsets: *const c_void, m: u64, nvotes: u64,
                               d_cert_words: *mut c_void, d_bad_words: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn nwc_dev_verify_batch_straus(d_digests: *const c_void, d_offsets: *const c_void, d_msg_index: *const c_void,
                                       m: u64, nvotes: u64, d_pks: *const c_void, d_sigs: *const c_void,
                                       d_leaf_words: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn nwc_dev_verify_batch_msm(d_digests: *const c_void, d_offsets: *const c_void, d_msg_index: *const c_void,
                                       m: u64, nvotes: u64, d_pks: *const c_void, d_sigs: *const c_void,
                                       d_leaf_words: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn nwc_msm_stats(groups_passed: *mut u64, groups_failed: *mut u64, key_overflows: *mut u64,
                         groups_skipped: *mut u64) -> c_int;
    pub fn nwc_dev_sha512_trunc32(d_data: *const c_void, d_offsets: *const c_void, n: u64, d_out32: *mut c_void,
                                  stream: *mut c_void) -> c_int;
    pub fn nwc_dev_sha512_trunc32_ranges(d_data: *const c_void, d_starts: *const c_void, d_ends: *const c_void, n: u64,
                                         d_out32: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn nwc_dev_derive32(tag: *const u8, taglen: c_int, first: u64, n: u64, d_out: *mut c_void,
                            stream: *mut c_void) -> c_int;
    pub fn nwc_dev_keygen_sign(d_seeds: *const c_void, d_msgs: *const c_void, n: u64, d_pks: *mut c_void,
                               d_sigs: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn nwc_dev_set_device(device: c_int) -> c_int;

    pub fn nwc_shard_bounds(n: u64, world: u32, rank: u32, lo: *mut u64, hi: *mut u64) -> c_int;
    pub fn nwc_cert_cuts(offsets: *const u32, m: usize, world: u32, cuts: *mut u64) -> c_int;
}
