//! src/validation/impls/slot_collector.rs -- the per-slot collector in front of
//! the HIP batch backend (`src/crypto/impls/hip.rs`).
//!
//! Reference call site: `HotstuffOperatorCommittee::sign` (src/validation/impls/hotstuff.rs:141-169)
//! ends every committee's duty with ONE `ThresholdSignature::new(t).threshold_aggregate(..)`
//! (:165-166).  Thousands of committees reach that line in the same slot, each with a handful of
//! shares -- far too little work for one GPU call.  With `--features hip` (rust/patches/0002-...)
//! the committee instead submits its job here and awaits a oneshot reply; one collector task
//! gathers the jobs of an aggregation window and runs them as one
//! `GenericThresholdSignature::threshold_aggregate_batch` per distinct threshold on a blocking
//! thread (the engine call is synchronous and owns the GPU context).
//!
//! A batch closes when `max_jobs` are pending or the window (started by its first job) expires.
//! Every job's result is exactly the reference's per-job `threshold_aggregate` result
//! (generic_threshold.rs:132-175, error order included): batching changes when, not what.
//! Mirrors `safestakeoperator_amd/collector.py` (`SlotCollector`), which the CPU and GPU tests of
//! the engine repository exercise (`tests/test_collector.py`); this file is type-checked by
//! inspection only (no cargo in the engine's build image).
//!
//! Knobs (environment, read once): `SSB_COLLECT_MAX_JOBS` (default 4096, the C2 batch of
//! BASELINE.json), `SSB_COLLECT_WINDOW_US` (default 5000).
use std::collections::HashMap;
use std::time::Duration;

use bls::{Hash256, PublicKey, Signature};
use lazy_static::lazy_static;
use log::error;
use tokio::sync::{mpsc, oneshot};
use tokio::time::{timeout_at, Instant};

use crate::crypto::generic_threshold::ThresholdJob;
use crate::crypto::ThresholdSignature;
use crate::utils::error::DvfError;

/// One committee's job, owned so it can cross into the collector task.
pub struct OwnedJob {
    pub sigs: Vec<Signature>,
    pub pks: Vec<PublicKey>,
    pub ids: Vec<u64>,
    pub msg: Hash256,
}

type Reply = oneshot::Sender<Result<Signature, DvfError>>;

struct Pending {
    t: usize,
    job: OwnedJob,
    reply: Reply,
}

pub struct SlotCollector {
    tx: mpsc::Sender<Pending>,
}

fn env_or<T: std::str::FromStr>(name: &str, default: T) -> T {
    std::env::var(name).ok().and_then(|v| v.parse().ok()).unwrap_or(default)
}

lazy_static! {
    /// The process's collector.  First touched from `HotstuffOperatorCommittee::sign`, i.e. inside
    /// the validator client's tokio runtime, which `tokio::spawn` below needs.
    pub static ref SLOT_COLLECTOR: SlotCollector = SlotCollector::spawn(
        env_or("SSB_COLLECT_MAX_JOBS", 4096usize),
        Duration::from_micros(env_or("SSB_COLLECT_WINDOW_US", 5000u64)),
    );
}

fn collector_gone() -> DvfError {
    DvfError::UnexpectedCall(String::from("slot collector stopped"))
}

impl SlotCollector {
    /// Starts the collector task on the current tokio runtime.
    pub fn spawn(max_jobs: usize, window: Duration) -> Self {
        let max_jobs = max_jobs.max(1);
        let (tx, rx) = mpsc::channel(4 * max_jobs);
        tokio::spawn(run(rx, max_jobs, window));
        Self { tx }
    }

    /// Drop-in for `ThresholdSignature::new(t).threshold_aggregate(sigs, pks, ids, msg)`
    /// (hotstuff.rs:165-166): same arguments, same `Result`, awaited instead of called.
    pub async fn threshold_aggregate(&self, t: usize, sigs: &[&Signature], pks: &[&PublicKey], ids: &[u64],
                                     msg: Hash256) -> Result<Signature, DvfError> {
        let job = OwnedJob {
            sigs: sigs.iter().map(|s| (*s).clone()).collect(),
            pks: pks.iter().map(|p| (*p).clone()).collect(),
            ids: ids.to_vec(),
            msg,
        };
        let (reply, rx) = oneshot::channel();
        self.tx.send(Pending { t, job, reply }).await.map_err(|_| collector_gone())?;
        rx.await.map_err(|_| collector_gone())?
    }
}

/// Collector task: one window at a time; the next window's jobs queue in the channel while the
/// current batch is on the GPU.
async fn run(mut rx: mpsc::Receiver<Pending>, max_jobs: usize, window: Duration) {
    loop {
        let first = match rx.recv().await {
            Some(p) => p,
            None => return, // every sender dropped
        };
        let deadline = Instant::now() + window;
        let mut batch = vec![first];
        while batch.len() < max_jobs {
            match timeout_at(deadline, rx.recv()).await {
                Ok(Some(p)) => batch.push(p),
                Ok(None) | Err(_) => break, // closed, or the window expired
            }
        }
        let mut by_t: HashMap<usize, Vec<Pending>> = HashMap::new();
        for p in batch {
            by_t.entry(p.t).or_default().push(p);
        }
        for (t, items) in by_t {
            // a committee whose sign() future was dropped no longer waits for its result
            let (jobs, replies): (Vec<OwnedJob>, Vec<Reply>) =
                items.into_iter().filter(|p| !p.reply.is_closed()).map(|p| (p.job, p.reply)).unzip();
            if jobs.is_empty() {
                continue;
            }
            match tokio::task::spawn_blocking(move || aggregate_owned(t, &jobs)).await {
                Ok(results) => {
                    for (reply, out) in replies.into_iter().zip(results) {
                        let _ = reply.send(out);
                    }
                }
                Err(e) => {
                    // engine panic (the reference's own `require` / `unwrap` panics included):
                    // every job of the batch sees it as an error instead of hanging
                    let msg = format!("threshold_aggregate_batch task failed: {}", e);
                    error!("{}", msg);
                    for reply in replies {
                        let _ = reply.send(Err(DvfError::UnexpectedCall(msg.clone())));
                    }
                }
            }
        }
    }
}

/// Borrowed `ThresholdJob`s over the owned jobs, then ONE batch call (the HIP backend's
/// `ssb_threshold_aggregate_batch`, or the generic per-job loop outside the engine's limits).
fn aggregate_owned(t: usize, jobs: &[OwnedJob]) -> Vec<Result<Signature, DvfError>> {
    let sig_refs: Vec<Vec<&Signature>> = jobs.iter().map(|j| j.sigs.iter().collect()).collect();
    let pk_refs: Vec<Vec<&PublicKey>> = jobs.iter().map(|j| j.pks.iter().collect()).collect();
    let borrowed: Vec<ThresholdJob> = jobs
        .iter()
        .enumerate()
        .map(|(i, j)| ThresholdJob { sigs: &sig_refs[i], pks: &pk_refs[i], ids: &j.ids, msg: j.msg })
        .collect();
    ThresholdSignature::new(t).threshold_aggregate_batch(&borrowed)
}
