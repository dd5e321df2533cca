//! `crypto_nwc`: the device side of Narwhal's `crypto` crate (/root/reference/crypto/src/lib.rs).
//!
//! The reference crate keeps its types and API; its verification bodies forward here
//!:
//!
//! ```ignore
//! // crypto/src/lib.rs:200-204  Signature::verify
//! pub fn verify(&self, digest: &Digest, public_key: &PublicKey) -> Result<(), CryptoError> {
//!     if crypto_nwc::verify_strict(&digest.0, &public_key.0, &self.flatten()) { Ok(()) }
//!     else { Err(CryptoError::new()) }
//! }
//! // crypto/src/lib.rs:206-219  Signature::verify_batch
//! pub fn verify_batch<'a, I>(digest: &Digest, votes: I) -> Result<(), CryptoError>
//! where I: IntoIterator<Item = &'a (PublicKey, Signature)> {
//!     let (pks, sigs): (Vec<[u8; 32]>, Vec<[u8; 64]>) =
//!         votes.into_iter().map(|(k, s)| (k.0, s.flatten())).unzip();
//!     if crypto_nwc::verify_batch(&digest.0, &pks, &sigs) { Ok(()) } else { Err(CryptoError::new()) }
//! }
//! // worker/src/processor.rs:38
//! let digest = Digest(crypto_nwc::digest32(&batch));
//! ```
//!
//! Return convention of the C ABI: 0 = valid, 1 = invalid, < 0 = device/runtime failure, which
//! is never reported as an invalid signature -- these wrappers panic on it, as the crate's
//! callers have no error path for a broken device.
mod ffi;

pub use ffi::*;

use std::ffi::CStr;
use std::os::raw::c_int;
use std::sync::Once;

static INIT: Once = Once::new();

/// `nwc_init(device_mask)` once per process (node start-up, node/src/main.rs:69-134).  Later
/// calls are no-ops; the wrappers below call it with mask 0 (device 0) if nobody did.
pub fn init(device_mask: u32) {
    INIT.call_once(|| {
        let rc = unsafe { ffi::nwc_init(device_mask) };
        check(rc);
    });
}

/// The hash of the sources and flags the linked libnwc.so was compiled from (nwc_build_id):
/// build.rs compiles with the repository's recipe (narwhal_amd/build.py --hipcc-args), so this
/// equals `python3 narwhal_amd/build.py --source-id` of the same tree; "unknown" for other builds.
pub fn build_id() -> String {
    unsafe { CStr::from_ptr(ffi::nwc_build_id()) }.to_string_lossy().into_owned()
}

fn check(rc: c_int) -> bool {
    if rc < 0 {
        let msg = unsafe { CStr::from_ptr(ffi::nwc_last_error()) };
        panic!("libnwc failure {}: {}", rc, msg.to_string_lossy());
    }
    rc == 0
}

/// `Signature::verify` = dalek `verify_strict` (crypto/src/lib.rs:200-204).
pub fn verify_strict(digest: &[u8; 32], public_key: &[u8; 32], signature: &[u8; 64]) -> bool {
    init(0);
    check(unsafe { ffi::nwc_verify_strict(digest.as_ptr(), public_key.as_ptr(), signature.as_ptr()) })
}

/// `Signature::verify_batch` = dalek `verify_batch` over one digest (crypto/src/lib.rs:206-219).
/// An empty batch is valid.
pub fn verify_batch(digest: &[u8; 32], public_keys: &[[u8; 32]], signatures: &[[u8; 64]]) -> bool {
    assert_eq!(public_keys.len(), signatures.len());
    init(0);
    let pks: Vec<u8> = public_keys.iter().flat_map(|k| k.iter().copied()).collect();
    let sigs: Vec<u8> = signatures.iter().flat_map(|s| s.iter().copied()).collect();
    check(unsafe {
        ffi::nwc_verify_batch(digest.as_ptr(), pks.as_ptr(), sigs.as_ptr(), public_keys.len(), std::ptr::null_mut())
    })
}

/// Many certificates at once (certificate c = `digests[c]` over votes `offsets[c]..offsets[c+1]`):
/// per-certificate verdicts and the bad-vote set.  `dalek_batch = false`: the exact per-vote leaves
/// (deterministic; Err on dalek's randomized domain); `true`: dalek's batch semantics -- each
/// certificate passes iff dalek's random-linear-combination equation holds for it: the comb-path
/// leaves for every vote, then the equation once per certificate over the votes they rejected
/// (exact in the 8-torsion group; the committee's repeated keys give the comb path without
/// `set_committee`), or, where no key combs apply, a Pippenger MSM per group of votes with the
/// leaves for the groups it rejects.  Each vote meets at most one random equation.  Returns
/// (certificate ok, vote bad) as bitmaps.
pub fn verify_batch_many(digests: &[[u8; 32]], offsets: &[u32], public_keys: &[[u8; 32]], signatures: &[[u8; 64]],
                         dalek_batch: bool) -> (Vec<u8>, Vec<u8>) {
    let m = digests.len();
    assert_eq!(offsets.len(), m + 1);
    assert_eq!(public_keys.len(), signatures.len());
    assert_eq!(offsets[m] as usize, public_keys.len());
    init(0);
    let dg: Vec<u8> = digests.iter().flat_map(|d| d.iter().copied()).collect();
    let pks: Vec<u8> = public_keys.iter().flat_map(|k| k.iter().copied()).collect();
    let sigs: Vec<u8> = signatures.iter().flat_map(|s| s.iter().copied()).collect();
    let mut ok = vec![0u8; (m + 7) / 8];
    let mut bad = vec![0u8; (public_keys.len() + 7) / 8];
    let f = if dalek_batch { ffi::nwc_verify_batch_msm_many } else { ffi::nwc_verify_batch_many };
    let rc = unsafe { f(dg.as_ptr(), offsets.as_ptr(), pks.as_ptr(), sigs.as_ptr(), m, ok.as_mut_ptr(), bad.as_mut_ptr()) };
    assert!(rc == 0, "libnwc failure {}", rc);
    (ok, bad)
}

/// `Sha512::digest(bytes)[..32]` (worker/src/processor.rs:38).
pub fn digest32(data: &[u8]) -> [u8; 32] {
    init(0);
    let mut out = [0u8; 32];
    check(unsafe { ffi::nwc_digest32(data.as_ptr(), data.len(), out.as_mut_ptr()) });
    out
}

/// The committee's keys (config/src/lib.rs:154-156), cached on the devices.  Optional: verdicts
/// never depend on it.
pub fn set_committee(public_keys: &[[u8; 32]]) {
    init(0);
    let pks: Vec<u8> = public_keys.iter().flat_map(|k| k.iter().copied()).collect();
    check(unsafe { ffi::nwc_set_committee(pks.as_ptr(), public_keys.len()) });
}

/// The worker's grouped batch digests (worker/src/processor.rs:35-55): a libnwc digester whose
/// drain thread hashes whatever has queued up (up to `max_group` batches, or what arrived within
/// `max_wait_us` of the first) in one GPU launch.  Batches are borrowed until their digest comes
/// back, so the queue owns them here and hands each back with its digest, in submission order.
pub struct BatchDigester {
    q: *mut ffi::nwc_digester,
    next_tag: u64,
    held: std::collections::VecDeque<(u64, Vec<u8>)>,
}

unsafe impl Send for BatchDigester {}

impl BatchDigester {
    pub fn new(max_group: u32, max_wait_us: u32) -> Self {
        init(0);
        let q = unsafe { ffi::nwc_digester_create(max_group, max_wait_us) };
        if q.is_null() {
            let msg = unsafe { CStr::from_ptr(ffi::nwc_last_error()) };
            panic!("libnwc digester: {}", msg.to_string_lossy());
        }
        BatchDigester { q, next_tag: 0, held: std::collections::VecDeque::new() }
    }

    /// Queue a batch (the Processor's `rx_batch.recv()`); it comes back from `next`.
    pub fn submit(&mut self, batch: Vec<u8>) {
        let tag = self.next_tag;
        self.next_tag += 1;
        check(unsafe { ffi::nwc_digester_submit(self.q, batch.as_ptr(), batch.len(), tag) });
        self.held.push_back((tag, batch));   // the Vec's heap buffer does not move
    }

    /// The oldest outstanding batch with its digest, waiting up to `wait_us` (None on timeout).
    /// A batch whose group failed on the device comes back as `Err(batch)` -- the caller keeps
    /// it (to hash on the CPU, retry or drop) -- so `held` and the returned tags never diverge;
    /// the library's sticky error with nothing left to return panics like every device error.
    pub fn next(&mut self, wait_us: u32) -> Option<Result<([u8; 32], Vec<u8>), Vec<u8>>> {
        if self.held.is_empty() {
            return None;
        }
        let (mut tag, mut dig, mut n) = (0u64, [0u8; 32], 0usize);
        let rc = unsafe { ffi::nwc_digester_poll(self.q, 1, wait_us, &mut tag, dig.as_mut_ptr(), &mut n) };
        if n == 0 {
            check(rc);
            return None;
        }
        let (t, batch) = self.held.pop_front().unwrap();
        assert_eq!(t, tag, "digests come back in submission order");
        Some(if rc < 0 { Err(batch) } else { Ok((dig, batch)) })
    }
}

impl Drop for BatchDigester {
    fn drop(&mut self) {
        unsafe { ffi::nwc_digester_destroy(self.q) };
    }
}
