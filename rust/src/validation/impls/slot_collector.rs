//! src/validation/impls/slot_collector.rs -- the per-slot collector in front of the
//! MI355X engine: the library's native collector (`ssb_collector_*`, include/ssbls.h of the engine
//! repository; csrc/ssb_collector.hip).
//!
//! Reference call site: `HotstuffOperatorCommittee::sign` (src/validation/impls/hotstuff.rs:141-169)
//! ends every committee's duty with ONE `ThresholdSignature::new(t).threshold_aggregate(..)`
//! (:165-166).  Thousands of committees reach that line in the same slot, each with a handful of
//! shares.  With `--features hip` (rust/patches/0002-...) the committee instead awaits
//! `SLOT_COLLECTOR.threshold_aggregate(..)`: the job's bytes are copied straight into the library's
//! open window (lock-free, from the calling task's thread), the library closes a window at
//! `SSB_COLLECT_MAX_JOBS` jobs or after `SSB_COLLECT_WINDOW_US`, runs it as one
//! `ssb_threshold_aggregate_batch_cached_dev` batch with `SSB_COLLECT_IN_FLIGHT` windows on the
//! device at once, and completes each job's oneshot from its worker thread.  Public keys travel as
//! rows of the engine's decoded-key table: a committee's operator keys are registered when the
//! committee is built (rust/patches/0003-...: `OperatorCommittee::from_definition`,
//! src/validation/operator_committees.rs:13-30, reached from `DvfSigner::spawn`,
//! src/node/dvfcore.rs:144-235), and any key seen for the first time at submit is registered then.
//!
//! Every job's result is exactly the reference's per-job `threshold_aggregate` result
//! (generic_threshold.rs:132-175, error order included; the two DifferentLength checks run here,
//! the rest in the engine); invalid shares the reference's scan would have met are logged as it logs
//! them (:167).  Jobs outside the engine's limits (t > SSB_MAX_T, more than 64 shares) take the
//! reference's own per-job call.  Mirrors `safestakeoperator_amd/collector.py` (`SlotCollector` on
//! `NativeCollector`), which the engine repository's GPU tests exercise
//! (tests/test_gpu_collector.py); this file is type-checked by inspection only (no cargo in the
//! engine's build image).
use std::collections::HashMap;
use std::os::raw::{c_char, c_int, c_void};
use std::sync::RwLock;

use bls::{Hash256, PublicKey, Signature};
use lazy_static::lazy_static;
use tokio::sync::oneshot;

use crate::crypto::impls::hip::{log_invalid_shares, SSB_MAX_T};
use crate::crypto::ThresholdSignature;
use crate::utils::error::DvfError;

/// ssb_collector_submit's per-job share limit.
pub const MAX_JOB_SHARES: usize = 64;

#[repr(C)]
pub struct SsbCtx {
    _private: [u8; 0],
}
#[repr(C)]
pub struct SsbCollector {
    _private: [u8; 0],
}

/// `ssb_job_result` (include/ssbls.h).
#[repr(C)]
pub struct SsbJobResult {
    sig96: [u8; 96],
    err: [u64; 2],
    verdicts: u64,
    status: i32,
    rc: i32,
    n_shares: u32,
    done: u32,
}

type JobDoneFn = extern "C" fn(user: *mut c_void, result: *const SsbJobResult);

extern "C" {
    fn ssb_create(out: *mut *mut SsbCtx, device_ordinal: c_int) -> c_int;
    fn ssb_last_error(ctx: *const SsbCtx) -> *const c_char;
    fn ssb_collector_create(ctx: *mut SsbCtx, max_jobs: u32, max_shares: u32, window_us: u32, in_flight: c_int,
                            out: *mut *mut SsbCollector) -> c_int;
    fn ssb_collector_register_keys(col: *mut SsbCollector, n: usize, pk48: *const u8, out_index: *mut u32) -> c_int;
    fn ssb_collector_submit(col: *mut SsbCollector, t: u32, n: u32, sig96: *const u8, pk_index: *const u32,
                            ids: *const u64, root32: *const u8, result: *mut SsbJobResult, cb: Option<JobDoneFn>,
                            user: *mut c_void) -> c_int;
}

// ssbls.h status tags (DvfError variants, src/utils/error.rs:12-60)
const SSB_DVF_OK: i32 = 0;
const SSB_DVF_INSUFFICIENT_SIGNATURES: i32 = 2;
const SSB_DVF_INVALID_OPERATOR_ID: i32 = 3;
const SSB_DVF_INSUFFICIENT_VALID_SIGNATURES: i32 = 4;

fn env_or<T: std::str::FromStr>(name: &str, default: T) -> T {
    std::env::var(name).ok().and_then(|v| v.parse().ok()).unwrap_or(default)
}

fn engine_error(msg: String) -> DvfError {
    DvfError::UnexpectedCall(format!("ssbls collector: {}", msg))
}

pub struct SlotCollector {
    col: *mut SsbCollector,
    /// compressed operator key -> its row in the engine's decoded-key table
    rows: RwLock<HashMap<[u8; 48], u32>>,
}
// The collector's submit and key registration are thread-safe (include/ssbls.h); its context lives
// as long as the process and is used only through it.
unsafe impl Send for SlotCollector {}
unsafe impl Sync for SlotCollector {}

lazy_static! {
    /// The process's collector: its own engine context (device `SSB_DEVICE`, default 0) on
    /// one-stream pipeline slots.  Knobs, read once: `SSB_COLLECT_MAX_JOBS` (default 4096, the C2
    /// batch of BASELINE.json), `SSB_COLLECT_WINDOW_US` (default 5000), `SSB_COLLECT_IN_FLIGHT`
    /// (default 20).
    pub static ref SLOT_COLLECTOR: Result<SlotCollector, String> = SlotCollector::create(
        env_or("SSB_DEVICE", 0i32),
        env_or("SSB_COLLECT_MAX_JOBS", 4096u32),
        env_or("SSB_COLLECT_WINDOW_US", 5000u32),
        env_or("SSB_COLLECT_IN_FLIGHT", 20i32),
    );
}

/// One submitted job: the engine writes `result` in place, then calls `job_done` with this box.
struct Pending {
    result: SsbJobResult,
    reply: Option<oneshot::Sender<Result<Signature, DvfError>>>,
    t: usize,
    ids: Vec<u64>,
}

/// ssb_job_done_fn, on the library's worker thread: convert, log as the reference's scan, reply.
extern "C" fn job_done(user: *mut c_void, _result: *const SsbJobResult) {
    let _ = std::panic::catch_unwind(|| {
        // the box handed over at submit; the library does not touch `result` after this call
        let mut p: Box<Pending> = unsafe { Box::from_raw(user as *mut Pending) };
        let out = result_of(&p.result, p.t, &p.ids);
        if let Some(tx) = p.reply.take() {
            let _ = tx.send(out); // the committee's sign() may have been dropped: nothing to do
        }
    });
}

fn result_of(r: &SsbJobResult, t: usize, ids: &[u64]) -> Result<Signature, DvfError> {
    if r.rc != 0 {
        return Err(engine_error(format!("the job's batch failed ({})", r.rc)));
    }
    if r.status == SSB_DVF_OK || r.status == SSB_DVF_INSUFFICIENT_VALID_SIGNATURES {
        let verdicts: Vec<u8> = (0..ids.len()).map(|i| ((r.verdicts >> i) & 1) as u8).collect();
        log_invalid_shares(t, ids, &verdicts);
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

impl SlotCollector {
    fn create(device: i32, max_jobs: u32, window_us: u32, in_flight: i32) -> Result<Self, String> {
        let mut ctx: *mut SsbCtx = std::ptr::null_mut();
        let rc = unsafe { ssb_create(&mut ctx, device) };
        if rc != 0 || ctx.is_null() {
            return Err(format!("ssb_create(device {}) returned {}", device, rc));
        }
        let mut col: *mut SsbCollector = std::ptr::null_mut();
        let max_jobs = max_jobs.max(1);
        let rc = unsafe { ssb_collector_create(ctx, max_jobs, 16 * max_jobs, window_us, in_flight, &mut col) };
        if rc != 0 || col.is_null() {
            let msg = unsafe { std::ffi::CStr::from_ptr(ssb_last_error(ctx)) }.to_string_lossy().into_owned();
            return Err(format!("ssb_collector_create returned {}: {}", rc, msg));
        }
        Ok(Self { col, rows: RwLock::new(HashMap::new()) })
    }

    /// Enter keys into the engine's decoded-key table (a committee's operator keys, when it is
    /// built); returns their rows.  Keys already registered keep their rows.
    pub fn register_keys(&self, pks: &[PublicKey]) -> Result<Vec<u32>, DvfError> {
        let refs: Vec<&PublicKey> = pks.iter().collect();
        self.rows_of(&refs)
    }

    fn rows_of(&self, pks: &[&PublicKey]) -> Result<Vec<u32>, DvfError> {
        let keys: Vec<[u8; 48]> = pks.iter().map(|p| p.serialize()).collect();
        {
            let m = self.rows.read().map_err(|_| engine_error(String::from("key map poisoned")))?;
            if let Some(rows) = keys.iter().map(|k| m.get(k).copied()).collect::<Option<Vec<u32>>>() {
                return Ok(rows);
            }
        }
        let mut m = self.rows.write().map_err(|_| engine_error(String::from("key map poisoned")))?;
        let fresh: Vec<[u8; 48]> = keys.iter().filter(|k| !m.contains_key(*k)).copied().collect();
        if !fresh.is_empty() {
            let bytes: Vec<u8> = fresh.iter().flat_map(|k| k.iter().copied()).collect();
            let mut idx = vec![0u32; fresh.len()];
            let rc = unsafe { ssb_collector_register_keys(self.col, fresh.len(), bytes.as_ptr(), idx.as_mut_ptr()) };
            if rc != 0 {
                return Err(engine_error(format!("ssb_collector_register_keys returned {}", rc)));
            }
            for (k, i) in fresh.into_iter().zip(idx) {
                m.insert(k, i);
            }
        }
        Ok(keys.iter().map(|k| m[k]).collect())
    }

    /// Drop-in for `ThresholdSignature::new(t).threshold_aggregate(sigs, pks, ids, msg)`
    /// (hotstuff.rs:165-166): same arguments, same `Result`, awaited instead of called.
    pub async fn threshold_aggregate(&self, t: usize, sigs: &[&Signature], pks: &[&PublicKey], ids: &[u64],
                                     msg: Hash256) -> Result<Signature, DvfError> {
        // generic_threshold.rs:133-138, in the reference's order
        if sigs.len() != pks.len() {
            return Err(DvfError::DifferentLength { x: sigs.len(), y: pks.len() });
        }
        if sigs.len() != ids.len() {
            return Err(DvfError::DifferentLength { x: sigs.len(), y: ids.len() });
        }
        if t == 0 || t > SSB_MAX_T || sigs.len() > MAX_JOB_SHARES {
            // outside the engine's limits: the reference's own per-job call
            return ThresholdSignature::new(t).threshold_aggregate(sigs, pks, ids, msg);
        }
        let rows = self.rows_of(pks)?;
        let sig: Vec<u8> = sigs.iter().flat_map(|s| s.serialize().to_vec()).collect();
        let (tx, rx) = oneshot::channel();
        let raw = Box::into_raw(Box::new(Pending {
            result: SsbJobResult { sig96: [0u8; 96], err: [0; 2], verdicts: 0, status: 0, rc: 0, n_shares: 0, done: 0 },
            reply: Some(tx),
            t,
            ids: ids.to_vec(),
        }));
        // the library copies the job's bytes before returning; it owns `raw` until job_done
        let rc = unsafe {
            ssb_collector_submit(self.col, t as u32, sigs.len() as u32, sig.as_ptr(), rows.as_ptr(), ids.as_ptr(),
                                 msg.as_bytes().as_ptr(), &mut (*raw).result, Some(job_done), raw as *mut c_void)
        };
        if rc != 0 {
            drop(unsafe { Box::from_raw(raw) });
            return Err(engine_error(format!("ssb_collector_submit returned {}", rc)));
        }
        rx.await.map_err(|_| engine_error(String::from("collector stopped")))?
    }
}

/// `SLOT_COLLECTOR.threshold_aggregate`, or the engine's construction error as a DvfError.
pub async fn threshold_aggregate(t: usize, sigs: &[&Signature], pks: &[&PublicKey], ids: &[u64], msg: Hash256)
                                 -> Result<Signature, DvfError> {
    match &*SLOT_COLLECTOR {
        Ok(c) => c.threshold_aggregate(t, sigs, pks, ids, msg).await,
        Err(e) => Err(engine_error(e.clone())),
    }
}

/// Registration hook for `OperatorCommittee::from_definition` (patch 0003).
pub fn register_committee_keys(pks: &[PublicKey]) -> Result<Vec<u32>, DvfError> {
    match &*SLOT_COLLECTOR {
        Ok(c) => c.register_keys(pks),
        Err(e) => Err(engine_error(e.clone())),
    }
}
