//! src/crypto/impls/hip.rs -- the threshold-BLS backend on an AMD MI355X (gfx950): libssbls.so
//! through its C ABI (`include/ssbls.h` of the engine repository), linked by `build.rs`.
//!
//! Selected with `--features hip` (rust/patches/0001-...: `define_mod!(hip_threshold_implementations,
//! crate::crypto::impls::hip::types)` in src/crypto/mod.rs).  It replaces, for the hot path only:
//!   * `TThresholdSignature::unsafe_aggregate` (impls/blst.rs:67-87) -> `ssb_unsafe_aggregate_batch`;
//!   * the new `TThresholdSignature::threshold_aggregate_batch` -> the process's collector: verify
//!     every share (RLC batch with the library's own secret 64-bit scalars, exact group tests on
//!     failure), the reference's scan and error order (generic_threshold.rs:132-175), Lagrange
//!     combine, compressed output -- the jobs join the windows every other caller fills.
//! `GenericThresholdSignature::threshold_aggregate` (one job) keeps its own loop: lighthouse verify
//! per share, then `unsafe_aggregate` here.
//!
//! ONE engine per process ([`ENGINE`]): one `ssb_ctx` (device streams, workspaces, the decoded-key
//! table) and one collector on it (`ssb_collector_create2`, wire records enabled).  This module's
//! batch calls, the per-slot collector of the validation path (src/validation/impls/slot_collector.rs)
//! and key registration all use it; the library serialises calls on a context (include/ssbls.h:
//! every entry point takes the context's lock), so no Rust-side lock guards it.  Hardware queues:
//! the process must export GPU_MAX_HW_QUEUES >= SSB_COLLECT_IN_FLIGHT + 1 (at most 32) before its
//! first HIP call -- HIP's default is 4, and the collector lowers `in_flight` to fit.
use std::collections::HashMap;
use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_void};
use std::sync::{mpsc, RwLock};

use bls::{Hash256, PublicKey, Signature};
use lazy_static::lazy_static;
use log::error;

use crate::crypto::generic_threshold::{TThresholdSignature, ThresholdJob};
use crate::utils::error::{require, DvfError};

/// The DST of impls/blst.rs:11 (proof-of-possession ciphersuite).
pub const DST: &[u8] = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
/// SSB_MAX_T of ssbls.h: larger thresholds run the generic per-job loop.
pub const SSB_MAX_T: usize = 64;
/// ssb_collector_submit's per-job share limit.
pub const MAX_JOB_SHARES: usize = 64;
/// bincode(bls::Signature): u64 length 194, "0x", 192 hex digits.
pub const WIRE_RECORD: usize = 202;

/// Provides the externally-facing, core BLS types.
pub mod types {
    pub use super::HipThresholdSignature as ThresholdSignature;
}

#[repr(C)]
pub struct SsbCtx {
    _private: [u8; 0],
}
#[repr(C)]
pub struct SsbCollector {
    _private: [u8; 0],
}
#[repr(C)]
pub struct SsbSigner {
    _private: [u8; 0],
}

/// `ssb_sign_result` (include/ssbls.h).
#[repr(C)]
pub struct SsbSignResult {
    pub sig96: [u8; 96],
    pub rc: i32,
    pub done: u32,
}

pub type SignDoneFn = extern "C" fn(user: *mut c_void, result: *const SsbSignResult);

/// `ssb_job_result` (include/ssbls.h).
#[repr(C)]
pub struct SsbJobResult {
    pub sig96: [u8; 96],
    pub err: [u64; 2],
    pub verdicts: u64,
    pub status: i32,
    pub rc: i32,
    pub n_shares: u32,
    pub done: u32,
    pub absent: u64,
}

impl SsbJobResult {
    pub fn new() -> Self {
        Self { sig96: [0u8; 96], err: [0; 2], verdicts: 0, status: 0, rc: 0, n_shares: 0, done: 0, absent: 0 }
    }
}

pub type JobDoneFn = extern "C" fn(user: *mut c_void, result: *const SsbJobResult);

extern "C" {
    fn ssb_create(out: *mut *mut SsbCtx, device_ordinal: c_int) -> c_int;
    fn ssb_last_error(ctx: *const SsbCtx) -> *const c_char;
    fn ssb_unsafe_aggregate_batch(
        ctx: *mut SsbCtx, n_jobs: usize, share_off: *const u32, sig96: *const u8, ids: *const u64, out_sig96: *mut u8,
        out_status: *mut i32,
    ) -> c_int;
    fn ssb_collector_create2(ctx: *mut SsbCtx, max_jobs: u32, max_shares: u32, window_us: u32, in_flight: c_int,
                             flags: u32, out: *mut *mut SsbCollector) -> c_int;
    fn ssb_collector_register_keys(col: *mut SsbCollector, n: usize, pk48: *const u8, out_index: *mut u32) -> c_int;
    fn ssb_collector_submit(col: *mut SsbCollector, t: u32, n: u32, sig96: *const u8, pk_index: *const u32,
                            ids: *const u64, root32: *const u8, result: *mut SsbJobResult, cb: Option<JobDoneFn>,
                            user: *mut c_void) -> c_int;
    fn ssb_collector_submit_wire(col: *mut SsbCollector, t: u32, n: u32, wire: *const *const u8, wire_len: *const usize,
                                 pk_index: *const u32, ids: *const u64, root32: *const u8, result: *mut SsbJobResult,
                                 cb: Option<JobDoneFn>, user: *mut c_void) -> c_int;
    fn ssb_collector_flush(col: *mut SsbCollector) -> c_int;
    fn ssb_signer_create(ctx: *mut SsbCtx, max_jobs: u32, window_us: u32, out: *mut *mut SsbSigner) -> c_int;
    fn ssb_signer_submit(s: *mut SsbSigner, sk32le: *const u8, root32: *const u8, result: *mut SsbSignResult,
                         cb: Option<SignDoneFn>, user: *mut c_void) -> c_int;
}

const SSB_COLLECTOR_WIRE: u32 = 1;
// ssbls.h status tags (DvfError variants, src/utils/error.rs:12-60)
const SSB_DVF_OK: i32 = 0;
const SSB_DVF_INSUFFICIENT_SIGNATURES: i32 = 2;
const SSB_DVF_INVALID_OPERATOR_ID: i32 = 3;
const SSB_DVF_INSUFFICIENT_VALID_SIGNATURES: i32 = 4;

fn env_or<T: std::str::FromStr>(name: &str, default: T) -> T {
    std::env::var(name).ok().and_then(|v| v.parse().ok()).unwrap_or(default)
}

pub fn engine_error(msg: String) -> DvfError {
    DvfError::UnexpectedCall(format!("ssbls: {}", msg))
}

/// The process's engine: its context, the collector and the local-signing window on it, and the
/// compressed-key -> table-row map.
pub struct Engine {
    ctx: *mut SsbCtx,
    col: *mut SsbCollector,
    signer: *mut SsbSigner,
    rows: RwLock<HashMap<[u8; 48], u32>>,
}
// The library serialises every call on the context, and the collector's submit and key registration
// are thread-safe (include/ssbls.h); both live as long as the process.
unsafe impl Send for Engine {}
unsafe impl Sync for Engine {}

lazy_static! {
    /// Created on first use: device `SSB_DEVICE` (default 0), collector knobs read once --
    /// `SSB_COLLECT_MAX_JOBS` (default 4096, the C2 batch of BASELINE.json), `SSB_COLLECT_WINDOW_US`
    /// (default 5000), `SSB_COLLECT_IN_FLIGHT` (default 20) -- and the signing window's
    /// `SSB_SIGN_MAX_JOBS` (default 4096) and `SSB_SIGN_WINDOW_US` (default 1000).
    pub static ref ENGINE: Result<Engine, String> = Engine::create(
        env_or("SSB_DEVICE", 0i32),
        env_or("SSB_COLLECT_MAX_JOBS", 4096u32),
        env_or("SSB_COLLECT_WINDOW_US", 5000u32),
        env_or("SSB_COLLECT_IN_FLIGHT", 20i32),
        env_or("SSB_SIGN_MAX_JOBS", 4096u32),
        env_or("SSB_SIGN_WINDOW_US", 1000u32),
    );
}

/// The process's engine, or its construction error as a DvfError.
pub fn engine() -> Result<&'static Engine, DvfError> {
    ENGINE.as_ref().map_err(|e| engine_error(e.clone()))
}

/// Where a job's result goes when the library's worker thread completes it.
pub enum Reply {
    Async(tokio::sync::oneshot::Sender<Result<Signature, DvfError>>),
    /// the wire path: the result with the job's absent-share mask (bit i: share i's record did not
    /// deserialize, so the reference would not have had operator i's signature at all)
    AsyncWire(tokio::sync::oneshot::Sender<Result<(Signature, u64), DvfError>>),
    Blocking(mpsc::Sender<(usize, Result<Signature, DvfError>)>, usize),
}

/// One submitted job: the engine writes `result` in place, then calls `job_done` with this box.
struct Pending {
    result: SsbJobResult,
    reply: Option<Reply>,
    t: usize,
    ids: Vec<u64>,
}

/// ssb_job_done_fn, on the library's worker thread: convert, log as the reference's scan, reply.
extern "C" fn job_done(user: *mut c_void, _result: *const SsbJobResult) {
    let _ = std::panic::catch_unwind(|| {
        // the box handed over at submit; the library does not touch `result` after this call
        let mut p: Box<Pending> = unsafe { Box::from_raw(user as *mut Pending) };
        let out = result_of(&p.result, p.t, &p.ids);
        match p.reply.take() {
            Some(Reply::Async(tx)) => {
                let _ = tx.send(out); // the committee's sign() may have been dropped: nothing to do
            }
            Some(Reply::AsyncWire(tx)) => {
                let absent = p.result.absent;
                let _ = tx.send(out.map(|s| (s, absent)));
            }
            Some(Reply::Blocking(tx, j)) => {
                let _ = tx.send((j, out));
            }
            None => {}
        }
    });
}

/// The job's `threshold_aggregate` result from its ssb_job_result.  Shares the wire path found
/// absent (a record that did not deserialize) are not in the reference's lists, so they are left
/// out of the scan's log as the reference never saw them.
fn result_of(r: &SsbJobResult, t: usize, ids: &[u64]) -> Result<Signature, DvfError> {
    if r.rc != 0 {
        return Err(engine_error(format!("the job's batch failed ({})", r.rc)));
    }
    if r.status == SSB_DVF_OK || r.status == SSB_DVF_INSUFFICIENT_VALID_SIGNATURES {
        let present: Vec<usize> = (0..ids.len()).filter(|i| (r.absent >> i) & 1 == 0).collect();
        let pids: Vec<u64> = present.iter().map(|&i| ids[i]).collect();
        let verdicts: Vec<u8> = present.iter().map(|&i| ((r.verdicts >> i) & 1) as u8).collect();
        log_invalid_shares(t, &pids, &verdicts);
    }
    match r.status {
        SSB_DVF_OK => Signature::deserialize(&r.sig96).map_err(DvfError::from),
        SSB_DVF_INSUFFICIENT_SIGNATURES => {
            Err(DvfError::InsufficientSignatures { got: r.err[0] as usize, expected: r.err[1] as usize })
        }
        SSB_DVF_INVALID_OPERATOR_ID => Err(DvfError::InvalidOperatorId { id: r.err[0] }),
        SSB_DVF_INSUFFICIENT_VALID_SIGNATURES => {
            Err(DvfError::InsufficientValidSignatures { got: r.err[0] as usize, expected: r.err[1] as usize })
        }
        s => Err(engine_error(format!("unexpected job status {}", s))),
    }
}

/// A job's shares as the collector takes them: compressed signatures, or the wire records received.
pub enum Shares<'a> {
    Compressed(&'a [&'a Signature]),
    Wire(&'a [&'a [u8]]),
}

/// One submitted signature: the library writes `result` in place, then calls `sign_done` with this box.
struct PendingSign {
    result: SsbSignResult,
    reply: Option<tokio::sync::oneshot::Sender<Result<Signature, DvfError>>>,
}

/// ssb_sign_done_fn, on the signing window's worker thread.
extern "C" fn sign_done(user: *mut c_void, _result: *const SsbSignResult) {
    let _ = std::panic::catch_unwind(|| {
        let mut p: Box<PendingSign> = unsafe { Box::from_raw(user as *mut PendingSign) };
        let out = if p.result.rc == 0 {
            Signature::deserialize(&p.result.sig96).map_err(DvfError::from)
        } else {
            Err(engine_error(format!("ssb_sign_batch failed ({})", p.result.rc)))
        };
        if let Some(tx) = p.reply.take() {
            let _ = tx.send(out); // the duty task may have been dropped: nothing to do
        }
    });
}

impl Engine {
    fn create(device: i32, max_jobs: u32, window_us: u32, in_flight: i32, sign_jobs: u32, sign_window_us: u32)
              -> Result<Self, String> {
        let mut ctx: *mut SsbCtx = std::ptr::null_mut();
        let rc = unsafe { ssb_create(&mut ctx, device) };
        if rc != 0 || ctx.is_null() {
            return Err(format!("ssb_create(device {}) returned {}", device, rc));
        }
        let mut col: *mut SsbCollector = std::ptr::null_mut();
        let max_jobs = max_jobs.max(1);
        let rc = unsafe {
            ssb_collector_create2(ctx, max_jobs, 16 * max_jobs, window_us, in_flight, SSB_COLLECTOR_WIRE, &mut col)
        };
        if rc != 0 || col.is_null() {
            return Err(format!("ssb_collector_create2 returned {}: {}", rc, last_error(ctx)));
        }
        let mut signer: *mut SsbSigner = std::ptr::null_mut();
        let rc = unsafe { ssb_signer_create(ctx, sign_jobs.max(1), sign_window_us, &mut signer) };
        if rc != 0 || signer.is_null() {
            return Err(format!("ssb_signer_create returned {}", rc));
        }
        Ok(Self { ctx, col, signer, rows: RwLock::new(HashMap::new()) })
    }

    /// `SecretKey::sign(msg)` into the signing window; `reply` receives the signature.  The key's
    /// bytes (big-endian from lighthouse, little-endian for the library) are wiped after the copy.
    pub fn sign_submit(&self, sk: &bls::SecretKey, msg: Hash256,
                       reply: tokio::sync::oneshot::Sender<Result<Signature, DvfError>>) -> Result<(), DvfError> {
        let mut le = [0u8; 32];
        {
            let be = sk.serialize();
            for (i, b) in be.as_bytes().iter().enumerate() {
                le[31 - i] = *b;
            }
        }
        let raw = Box::into_raw(Box::new(PendingSign {
            result: SsbSignResult { sig96: [0u8; 96], rc: 0, done: 0 },
            reply: Some(reply),
        }));
        let rc = unsafe {
            ssb_signer_submit(self.signer, le.as_ptr(), msg.as_bytes().as_ptr(), &mut (*raw).result, Some(sign_done),
                              raw as *mut c_void)
        };
        for b in le.iter_mut() {
            unsafe { std::ptr::write_volatile(b, 0) };
        }
        if rc != 0 {
            drop(unsafe { Box::from_raw(raw) });
            return Err(engine_error(format!("ssb_signer_submit returned {}", rc)));
        }
        Ok(())
    }

    /// Table rows of these keys if every one is registered already (no library call).
    pub fn known_rows(&self, pks: &[&PublicKey]) -> Option<Vec<u32>> {
        let m = self.rows.read().ok()?;
        pks.iter().map(|p| m.get(&p.serialize()).copied()).collect()
    }

    /// Enter keys into the engine's decoded-key table (a committee's operator keys, when it is
    /// built); returns their rows.  Keys already registered keep their rows.  Blocking (the keys'
    /// decode on the device): async callers use `spawn_blocking` or register at committee creation.
    pub fn rows_of(&self, pks: &[&PublicKey]) -> Result<Vec<u32>, DvfError> {
        if let Some(rows) = self.known_rows(pks) {
            return Ok(rows);
        }
        let keys: Vec<[u8; 48]> = pks.iter().map(|p| p.serialize()).collect();
        let mut m = self.rows.write().map_err(|_| engine_error(String::from("key map poisoned")))?;
        let fresh: Vec<[u8; 48]> = keys.iter().filter(|k| !m.contains_key(*k)).copied().collect();
        if !fresh.is_empty() {
            let bytes: Vec<u8> = fresh.iter().flat_map(|k| k.iter().copied()).collect();
            let mut idx = vec![0u32; fresh.len()];
            let rc = unsafe { ssb_collector_register_keys(self.col, fresh.len(), bytes.as_ptr(), idx.as_mut_ptr()) };
            if rc != 0 {
                return Err(engine_error(format!("ssb_collector_register_keys returned {}: {}", rc, last_error(self.ctx))));
            }
            for (k, i) in fresh.into_iter().zip(idx) {
                m.insert(k, i);
            }
        }
        Ok(keys.iter().map(|k| m[k]).collect())
    }

    /// One job into the collector's open window; `reply` receives its result.  The caller has done
    /// the reference's two DifferentLength checks and the engine's limits (t <= SSB_MAX_T, at most
    /// MAX_JOB_SHARES shares).
    pub fn submit(&self, t: usize, shares: Shares, rows: &[u32], ids: &[u64], msg: Hash256, reply: Reply)
                  -> Result<(), DvfError> {
        let raw = Box::into_raw(Box::new(Pending { result: SsbJobResult::new(), reply: Some(reply), t, ids: ids.to_vec() }));
        // the library copies the job's bytes before returning; it owns `raw` until job_done
        let rc = match shares {
            Shares::Compressed(sigs) => {
                let sig: Vec<u8> = sigs.iter().flat_map(|s| s.serialize().to_vec()).collect();
                unsafe {
                    ssb_collector_submit(self.col, t as u32, sigs.len() as u32, sig.as_ptr(), rows.as_ptr(), ids.as_ptr(),
                                         msg.as_bytes().as_ptr(), &mut (*raw).result, Some(job_done), raw as *mut c_void)
                }
            }
            Shares::Wire(recs) => {
                let ptrs: Vec<*const u8> = recs.iter().map(|r| r.as_ptr()).collect();
                let lens: Vec<usize> = recs.iter().map(|r| r.len()).collect();
                unsafe {
                    ssb_collector_submit_wire(self.col, t as u32, recs.len() as u32, ptrs.as_ptr(), lens.as_ptr(),
                                              rows.as_ptr(), ids.as_ptr(), msg.as_bytes().as_ptr(), &mut (*raw).result,
                                              Some(job_done), raw as *mut c_void)
                }
            }
        };
        if rc != 0 {
            drop(unsafe { Box::from_raw(raw) });
            return Err(engine_error(format!("ssb_collector_submit returned {}", rc)));
        }
        Ok(())
    }

    fn flush(&self) {
        unsafe { ssb_collector_flush(self.col) };
    }
}

fn last_error(c: *mut SsbCtx) -> String {
    unsafe { CStr::from_ptr(ssb_last_error(c)) }.to_string_lossy().into_owned()
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
        let e = engine().expect("ssbls engine");
        let rc = unsafe {
            ssb_unsafe_aggregate_batch(e.ctx, 1, off.as_ptr(), bytes.as_ptr(), ids.as_ptr(), out.as_mut_ptr(),
                                       status.as_mut_ptr())
        };
        assert_eq!(rc, 0, "ssb_unsafe_aggregate_batch: {}", last_error(e.ctx));
        // a share that does not decode: the reference's deserialize(..).unwrap() panics (blst.rs:84)
        assert_eq!(status[0], SSB_DVF_OK, "unsafe_aggregate: a share does not decode");
        Signature::deserialize(&out).unwrap()
    }

    fn threshold_aggregate(&self, _sigs: &[&Signature], _pks: &[&PublicKey], _msg: Hash256) -> Result<Signature, DvfError> {
        Err(DvfError::UnexpectedCall(String::from("threshold_aggregate")))
    }

    fn threshold_aggregate_batch(&self, jobs: &[ThresholdJob]) -> Option<Vec<Result<Signature, DvfError>>> {
        if self.t == 0 || self.t > SSB_MAX_T || jobs.iter().any(|j| j.sigs.len() > MAX_JOB_SHARES) {
            return None; // outside the engine's limits: GenericThresholdSignature's per-job loop
        }
        Some(aggregate_batch(self.t, jobs))
    }
}

/// `GenericThresholdSignature::threshold_aggregate` (generic_threshold.rs:132-175) for every job,
/// through the process's collector (the jobs share windows with every other caller), blocking until
/// all are done.  The two DifferentLength checks run here, in the reference's order; the rest --
/// InsufficientSignatures, InvalidOperatorId (only when reached before the t-th valid share),
/// duplicate ids skipped unverified, InsufficientValidSignatures, the combine -- is the engine's,
/// per job.  Shares the reference's scan would have verified and found invalid are logged as it
/// logs them (generic_threshold.rs:167).
pub fn aggregate_batch(t: usize, jobs: &[ThresholdJob]) -> Vec<Result<Signature, DvfError>> {
    let nj = jobs.len();
    let mut out: Vec<Option<Result<Signature, DvfError>>> = (0..nj).map(|_| None).collect();
    let e = match engine() {
        Ok(e) => e,
        Err(err) => return (0..nj).map(|_| Err(err.clone())).collect(),
    };
    let (tx, rx) = mpsc::channel();
    let mut waiting = 0usize;
    for (j, job) in jobs.iter().enumerate() {
        if job.sigs.len() != job.pks.len() {
            out[j] = Some(Err(DvfError::DifferentLength { x: job.sigs.len(), y: job.pks.len() }));
            continue;
        }
        if job.sigs.len() != job.ids.len() {
            out[j] = Some(Err(DvfError::DifferentLength { x: job.sigs.len(), y: job.ids.len() }));
            continue;
        }
        let submitted = e.rows_of(job.pks).and_then(|rows| {
            e.submit(t, Shares::Compressed(job.sigs), &rows, job.ids, job.msg, Reply::Blocking(tx.clone(), j))
        });
        match submitted {
            Ok(()) => waiting += 1,
            Err(err) => out[j] = Some(Err(err)),
        }
    }
    if waiting > 0 {
        e.flush(); // close the open window now: this caller waits for its jobs
    }
    for _ in 0..waiting {
        match rx.recv() {
            Ok((j, r)) => out[j] = Some(r),
            Err(_) => break,
        }
    }
    out.into_iter().map(|o| o.unwrap_or_else(|| Err(engine_error(String::from("collector stopped"))))).collect()
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
