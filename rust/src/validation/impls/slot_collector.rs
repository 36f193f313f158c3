//! src/validation/impls/slot_collector.rs -- the per-slot collector in front of the
//! MI355X engine: the library's native collector (`ssb_collector_*`, include/ssbls.h of the engine
//! repository; csrc/ssb_collector.hip) of the process's ONE engine (`crypto::impls::hip::ENGINE`,
//! shared with `HipThresholdSignature`'s batch calls and key registration).
//!
//! Reference call site: `HotstuffOperatorCommittee::sign` (src/validation/impls/hotstuff.rs:141-169)
//! ends every committee's duty with ONE `ThresholdSignature::new(t).threshold_aggregate(..)`
//! (:165-166).  Thousands of committees reach that line in the same slot, each with a handful of
//! shares.  With `--features hip` (rust/patches/0002-...) the committee instead awaits
//! [`threshold_aggregate_wire`]: the shares travel as the bytes the operators sent
//! (`TOperator::sign_wire`, rust/patches/0004-...: no `bincode::deserialize::<Signature>` -- a G2
//! decompression, an Fp2 square root -- per share on a tokio thread, operator.rs:108), the job's
//! bytes are copied straight into the library's open window (lock-free, from the calling task's
//! thread), the library closes a window at `SSB_COLLECT_MAX_JOBS` jobs or after
//! `SSB_COLLECT_WINDOW_US`, decodes and decompresses the records on the device and runs the window
//! as one `ssb_threshold_aggregate_batch_wire_cached_dev` batch with `SSB_COLLECT_IN_FLIGHT` windows
//! on the device at once, and completes each job's oneshot from its worker thread.  A record that
//! does not deserialize makes its share ABSENT -- exactly the reference, whose RemoteOperator::sign
//! drops it (`Err` after the retries, then `.flatten()`): the job's share count shrinks and
//! InsufficientSignatures can result.  Public keys travel as rows of the engine's decoded-key table:
//! a committee's operator keys are registered when the committee is built (rust/patches/0003-...:
//! `OperatorCommittee::from_definition`, src/validation/operator_committees.rs:13-30, reached from
//! `DvfSigner::spawn`, src/node/dvfcore.rs:144-235); a key first seen at submit is registered on a
//! blocking thread (`spawn_blocking`), never on the async worker.
//!
//! Every job's result is exactly the reference's per-job `threshold_aggregate` result
//! (generic_threshold.rs:132-175, error order included; the two DifferentLength checks run here,
//! the rest in the engine); invalid shares the reference's scan would have met are logged as it logs
//! them (:167).  Jobs outside the engine's limits (t > SSB_MAX_T, more than 64 shares) take the
//! reference's own per-job call.  Mirrors `safestakeoperator_amd/collector.py` (`NativeCollector`,
//! `SlotCollector`), which the engine repository's GPU tests exercise (tests/test_gpu_collector.py);
//! this file is type-checked by inspection only (no cargo in the engine's build image).
use bls::{Hash256, PublicKey, Signature};
use tokio::sync::oneshot;

use crate::crypto::impls::hip::{engine, engine_error, Engine, Reply, Shares, MAX_JOB_SHARES, SSB_MAX_T};
use crate::crypto::ThresholdSignature;
use crate::utils::error::DvfError;

/// Table rows of a job's keys: known rows at once, else registration on a blocking thread.
async fn rows(e: &'static Engine, pks: &[&PublicKey]) -> Result<Vec<u32>, DvfError> {
    if let Some(r) = e.known_rows(pks) {
        return Ok(r);
    }
    let owned: Vec<PublicKey> = pks.iter().map(|p| (*p).clone()).collect();
    tokio::task::spawn_blocking(move || {
        let refs: Vec<&PublicKey> = owned.iter().collect();
        e.rows_of(&refs)
    })
    .await
    .map_err(|_| engine_error(String::from("key registration task failed")))?
}

async fn submit_and_wait(e: &'static Engine, t: usize, shares: Shares<'_>, rows: &[u32], ids: &[u64], msg: Hash256)
                         -> Result<Signature, DvfError> {
    let (tx, rx) = oneshot::channel();
    e.submit(t, shares, rows, ids, msg, Reply::Async(tx))?;
    rx.await.map_err(|_| engine_error(String::from("collector stopped")))?
}

/// Drop-in for `ThresholdSignature::new(t).threshold_aggregate(sigs, pks, ids, msg)`
/// (hotstuff.rs:165-166): same arguments, same `Result`, awaited instead of called.
pub async fn threshold_aggregate(t: usize, sigs: &[&Signature], pks: &[&PublicKey], ids: &[u64], msg: Hash256)
                                 -> Result<Signature, DvfError> {
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
    let e = engine()?;
    let r = rows(e, pks).await?;
    submit_and_wait(e, t, Shares::Compressed(sigs), &r, ids, msg).await
}

/// The same with the shares as received: `records[i]` is operator `ids[i]`'s bincode(bls::Signature)
/// (`TOperator::sign_wire`).  A record that does not deserialize is absent from the job, as the
/// reference's RemoteOperator::sign drops it before threshold_aggregate (operator.rs:108-131,
/// hotstuff.rs:150-155): `sigs.len()` counts the records that deserialize.  Returns the combined
/// signature and the ids of the operators whose record deserialized -- the reference's `ids`
/// (hotstuff.rs:157, reported by signing_method.rs:337-338).
pub async fn threshold_aggregate_wire(t: usize, records: &[&[u8]], pks: &[&PublicKey], ids: &[u64], msg: Hash256)
                                      -> Result<(Signature, Vec<u64>), DvfError> {
    if records.len() != pks.len() {
        return Err(DvfError::DifferentLength { x: records.len(), y: pks.len() });
    }
    if records.len() != ids.len() {
        return Err(DvfError::DifferentLength { x: records.len(), y: ids.len() });
    }
    if t == 0 || t > SSB_MAX_T || records.len() > MAX_JOB_SHARES {
        // outside the engine's limits: deserialize on the CPU as the reference does, drop what fails
        let mut kept: Vec<(Signature, &PublicKey, u64)> = Vec::new();
        for ((r, p), id) in records.iter().zip(pks).zip(ids) {
            if let Ok(s) = bincode::deserialize::<Signature>(r) {
                kept.push((s, *p, *id));
            }
        }
        let sigs: Vec<&Signature> = kept.iter().map(|k| &k.0).collect();
        let kp: Vec<&PublicKey> = kept.iter().map(|k| k.1).collect();
        let ki: Vec<u64> = kept.iter().map(|k| k.2).collect();
        return ThresholdSignature::new(t).threshold_aggregate(&sigs, &kp, &ki, msg).map(|s| (s, ki));
    }
    let e = engine()?;
    let r = rows(e, pks).await?;
    let (tx, rx) = oneshot::channel();
    e.submit(t, Shares::Wire(records), &r, ids, msg, Reply::AsyncWire(tx))?;
    let (sig, absent) = rx.await.map_err(|_| engine_error(String::from("collector stopped")))??;
    let present = ids.iter().enumerate().filter(|(i, _)| (absent >> i) & 1 == 0).map(|(_, id)| *id).collect();
    Ok((sig, present))
}

/// Registration hook for `OperatorCommittee::from_definition` (patch 0003).
pub fn register_committee_keys(pks: &[PublicKey]) -> Result<Vec<u32>, DvfError> {
    let refs: Vec<&PublicKey> = pks.iter().collect();
    engine()?.rows_of(&refs)
}
