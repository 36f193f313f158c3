//! src/crypto/impls/hip.rs -- the threshold-BLS backend on an AMD MI355X (gfx950): libssbls.so
//! through its C ABI (`include/ssbls.h` of the engine repository), linked by `build.rs`.
//!
//! Selected with `--features hip` (rust/patches/0001-...: `define_mod!(hip_threshold_implementations,
//! crate::crypto::impls::hip::types)` in src/crypto/mod.rs).  It replaces, for the hot path only:
//!   * `TThresholdSignature::unsafe_aggregate` (impls/blst.rs:67-87) -> `ssb_unsafe_aggregate_batch`;
//!   * the new `TThresholdSignature::threshold_aggregate_batch` -> `ssb_threshold_aggregate_batch`:
//!     verify every share (RLC batch with the library's own secret 64-bit scalars, exact group
//!     tests on failure), the reference's scan and error order (generic_threshold.rs:132-175),
//!     Lagrange combine, compressed output -- one call for all of a slot's jobs.
//! `GenericThresholdSignature::threshold_aggregate` (one job) keeps its own loop: lighthouse verify
//! per share, then `unsafe_aggregate` here.
use std::collections::HashMap;
use std::ffi::CStr;
use std::os::raw::{c_char, c_int};
use std::sync::Mutex;

use bls::{Hash256, PublicKey, Signature};
use lazy_static::lazy_static;
use log::error;

use crate::crypto::generic_threshold::{TThresholdSignature, ThresholdJob};
use crate::utils::error::{require, DvfError};

/// The DST of impls/blst.rs:11 (proof-of-possession ciphersuite).
pub const DST: &[u8] = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
/// SSB_MAX_T of ssbls.h: larger thresholds run the generic per-job loop.
pub const SSB_MAX_T: usize = 64;

/// Provides the externally-facing, core BLS types.
pub mod types {
    pub use super::HipThresholdSignature as ThresholdSignature;
}

#[repr(C)]
pub struct SsbCtx {
    _private: [u8; 0],
}

extern "C" {
    fn ssb_create(out: *mut *mut SsbCtx, device_ordinal: c_int) -> c_int;
    fn ssb_destroy(ctx: *mut SsbCtx);
    fn ssb_last_error(ctx: *const SsbCtx) -> *const c_char;
    fn ssb_threshold_aggregate_batch(
        ctx: *mut SsbCtx, n_jobs: usize, share_off: *const u32, t: *const u32, sig96: *const u8, pk48: *const u8,
        ids: *const u64, job_root: *const u32, n_roots: usize, roots32: *const u8, dst: *const u8, dst_len: usize,
        rlc_seed: u64, out_sig96: *mut u8, out_status: *mut i32, out_err: *mut u64, share_verdicts: *mut u8,
    ) -> c_int;
    fn ssb_unsafe_aggregate_batch(
        ctx: *mut SsbCtx, n_jobs: usize, share_off: *const u32, sig96: *const u8, ids: *const u64, out_sig96: *mut u8,
        out_status: *mut i32,
    ) -> c_int;
}

// ssbls.h status tags (DvfError variants, src/utils/error.rs:12-60)
const SSB_DVF_OK: i32 = 0;
const SSB_DVF_INSUFFICIENT_SIGNATURES: i32 = 2;
const SSB_DVF_INVALID_OPERATOR_ID: i32 = 3;
const SSB_DVF_INSUFFICIENT_VALID_SIGNATURES: i32 = 4;

/// One engine context per process: it owns the device streams, the workspace and the decoded
/// tables.  A context must not be used by two threads at once, so the Mutex serialises the
/// callers (the per-slot collector calls from one `spawn_blocking` worker anyway).
struct Ctx(*mut SsbCtx);
// The raw context is only ever touched under CTX's lock.
unsafe impl Send for Ctx {}
impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { ssb_destroy(self.0) }
    }
}

lazy_static! {
    static ref CTX: Mutex<Option<Ctx>> = Mutex::new(None);
}

fn engine_error(msg: String) -> DvfError {
    DvfError::UnexpectedCall(format!("ssbls: {}", msg))
}

fn last_error(c: *mut SsbCtx) -> String {
    unsafe { CStr::from_ptr(ssb_last_error(c)) }.to_string_lossy().into_owned()
}

/// Runs `f` on the process's context, creating it on first use (device `SSB_DEVICE`, default 0).
fn with_ctx<R>(f: impl FnOnce(*mut SsbCtx) -> R) -> Result<R, DvfError> {
    let mut guard = CTX.lock().map_err(|_| engine_error(String::from("context lock poisoned")))?;
    if guard.is_none() {
        let device: c_int = std::env::var("SSB_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0);
        let mut p: *mut SsbCtx = std::ptr::null_mut();
        let rc = unsafe { ssb_create(&mut p, device) };
        if rc != 0 || p.is_null() {
            return Err(engine_error(format!("ssb_create(device {}) returned {}", device, rc)));
        }
        *guard = Some(Ctx(p));
    }
    Ok(f(guard.as_ref().unwrap().0))
}

#[derive(Clone)]
pub struct HipThresholdSignature {
    t: usize,
}

impl TThresholdSignature for HipThresholdSignature {
    fn infinity(threshold: usize) -> Self {
        Self { t: threshold }
    }

    fn threshold(&self) -> usize {
        self.t
    }

    /// impls/blst.rs:67-87: the first t shares, Lagrange coefficients of exactly t ids (the
    /// reference's `require` panics otherwise), 255-bit multiples summed from infinity.
    fn unsafe_aggregate(&self, sigs: &[&Signature], ids: &[u64]) -> Signature {
        require(ids.len() == self.t, "Different length");
        let bytes: Vec<u8> = sigs[..self.t].iter().flat_map(|s| s.serialize().to_vec()).collect();
        let off = [0u32, self.t as u32];
        let mut out = [0u8; 96];
        let mut status = [0i32; 1];
        let (rc, msg) = with_ctx(|c| {
            let rc = unsafe {
                ssb_unsafe_aggregate_batch(c, 1, off.as_ptr(), bytes.as_ptr(), ids.as_ptr(), out.as_mut_ptr(),
                                           status.as_mut_ptr())
            };
            (rc, if rc != 0 { last_error(c) } else { String::new() })
        })
        .expect("ssbls context");
        assert_eq!(rc, 0, "ssb_unsafe_aggregate_batch: {}", msg);
        // a share that does not decode: the reference's deserialize(..).unwrap() panics (blst.rs:84)
        assert_eq!(status[0], SSB_DVF_OK, "unsafe_aggregate: a share does not decode");
        Signature::deserialize(&out).unwrap()
    }

    fn threshold_aggregate(&self, _sigs: &[&Signature], _pks: &[&PublicKey], _msg: Hash256) -> Result<Signature, DvfError> {
        Err(DvfError::UnexpectedCall(String::from("threshold_aggregate")))
    }

    fn threshold_aggregate_batch(&self, jobs: &[ThresholdJob]) -> Option<Vec<Result<Signature, DvfError>>> {
        if self.t == 0 || self.t > SSB_MAX_T {
            return None; // outside the engine's limits: GenericThresholdSignature's per-job loop
        }
        Some(aggregate_batch(self.t, jobs))
    }
}

/// `GenericThresholdSignature::threshold_aggregate` (generic_threshold.rs:132-175) for every job,
/// in ONE engine call.  The two DifferentLength checks run here, in the reference's order; the
/// rest -- InsufficientSignatures, InvalidOperatorId (only when reached before the t-th valid
/// share), duplicate ids skipped unverified, InsufficientValidSignatures, the combine -- is the
/// engine's, per job.  Shares the reference's scan would have verified and found invalid are
/// logged as it logs them (generic_threshold.rs:167).
pub fn aggregate_batch(t: usize, jobs: &[ThresholdJob]) -> Vec<Result<Signature, DvfError>> {
    let nj = jobs.len();
    if nj == 0 {
        return Vec::new();
    }
    let mut out: Vec<Option<Result<Signature, DvfError>>> = (0..nj).map(|_| None).collect();
    let mut off: Vec<u32> = Vec::with_capacity(nj + 1);
    off.push(0);
    let (mut sig, mut pk, mut ids) = (Vec::<u8>::new(), Vec::<u8>::new(), Vec::<u64>::new());
    let mut roots: Vec<Hash256> = Vec::new();
    let mut root_index: HashMap<Hash256, u32> = HashMap::new();
    let (mut job_root, mut tt) = (Vec::<u32>::with_capacity(nj), Vec::<u32>::with_capacity(nj));
    for (j, job) in jobs.iter().enumerate() {
        if job.sigs.len() != job.pks.len() {
            out[j] = Some(Err(DvfError::DifferentLength { x: job.sigs.len(), y: job.pks.len() }));
        } else if job.sigs.len() != job.ids.len() {
            out[j] = Some(Err(DvfError::DifferentLength { x: job.sigs.len(), y: job.ids.len() }));
        }
        let n = if out[j].is_some() { 0 } else { job.sigs.len() };
        for i in 0..n {
            sig.extend_from_slice(&job.sigs[i].serialize());
            pk.extend_from_slice(&job.pks[i].serialize());
            ids.push(job.ids[i]);
        }
        off.push(ids.len() as u32);
        tt.push(t as u32);
        let next = roots.len() as u32;
        let r = *root_index.entry(job.msg).or_insert_with(|| {
            roots.push(job.msg);
            next
        });
        job_root.push(r);
    }
    let root_bytes: Vec<u8> = roots.iter().flat_map(|r| r.as_bytes().to_vec()).collect();
    let (mut osig, mut ost, mut oerr) = (vec![0u8; 96 * nj], vec![0i32; nj], vec![0u64; 2 * nj]);
    let mut verdicts = vec![0u8; ids.len().max(1)];
    let seed: u64 = rand::random(); // only XORed into the library's own getrandom() key
    let called = with_ctx(|c| {
        let rc = unsafe {
            ssb_threshold_aggregate_batch(c, nj, off.as_ptr(), tt.as_ptr(), sig.as_ptr(), pk.as_ptr(), ids.as_ptr(),
                                          job_root.as_ptr(), roots.len(), root_bytes.as_ptr(), DST.as_ptr(), DST.len(),
                                          seed, osig.as_mut_ptr(), ost.as_mut_ptr(), oerr.as_mut_ptr(),
                                          verdicts.as_mut_ptr())
        };
        if rc != 0 { Err(engine_error(format!("ssb_threshold_aggregate_batch returned {}: {}", rc, last_error(c)))) } else { Ok(()) }
    });
    if let Err(e) = called.and_then(|r| r) {
        return out.into_iter().map(|o| o.unwrap_or_else(|| Err(e.clone()))).collect();
    }
    (0..nj)
        .map(|j| {
            if let Some(r) = out[j].take() {
                return r;
            }
            let (b, e) = (off[j] as usize, off[j + 1] as usize);
            if ost[j] == SSB_DVF_OK || ost[j] == SSB_DVF_INSUFFICIENT_VALID_SIGNATURES {
                log_invalid_shares(t, &ids[b..e], &verdicts[b..e]);
            }
            match ost[j] {
                SSB_DVF_OK => Signature::deserialize(&osig[96 * j..96 * j + 96]).map_err(DvfError::from),
                SSB_DVF_INSUFFICIENT_SIGNATURES => Err(DvfError::InsufficientSignatures {
                    got: oerr[2 * j] as usize,
                    expected: oerr[2 * j + 1] as usize,
                }),
                SSB_DVF_INVALID_OPERATOR_ID => Err(DvfError::InvalidOperatorId { id: oerr[2 * j] }),
                SSB_DVF_INSUFFICIENT_VALID_SIGNATURES => Err(DvfError::InsufficientValidSignatures {
                    got: oerr[2 * j] as usize,
                    expected: oerr[2 * j + 1] as usize,
                }),
                s => Err(engine_error(format!("unexpected job status {}", s))),
            }
        })
        .collect()
}

/// The reference's scan order (generic_threshold.rs:149-169): shares up to the t-th accepted one,
/// ids already accepted skipped unverified; every verified-and-invalid share is logged.
pub(crate) fn log_invalid_shares(t: usize, ids: &[u64], verdicts: &[u8]) {
    let mut accepted: Vec<u64> = Vec::with_capacity(t);
    for (id, v) in ids.iter().zip(verdicts) {
        if accepted.contains(id) {
            continue;
        }
        if *v != 0 {
            accepted.push(*id);
            if accepted.len() >= t {
                break;
            }
        } else {
            error!("Invalid signature from operator {}", id);
        }
    }
}
