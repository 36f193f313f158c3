//! src/validation/impls/slot_signer.rs -- the local-signing window in front of the
//! MI355X engine: the library's `ssb_signer_*` (include/ssbls.h of the engine repository;
//! csrc/ssb_collector.hip) on the process's ONE engine (`crypto::impls::hip::ENGINE`).
//!
//! Reference call site: `DvfSigner::local_sign_and_store` (src/node/dvfcore.rs:245-251) signs every
//! duty's signing root with the operator's key share, `self.local_keypair.sk.sign(message)` (:241-243)
//! -- one hash_to_G2 and one G2 scalar multiplication on the duty's tokio task.  Every duty of every
//! validator the operator serves reaches it once per slot (src/validation/signing_method.rs:318:
//! attestations, blocks, aggregates, sync-committee messages, and the selection proofs and RANDAO
//! reveals every operator signs, :269-292).  With `--features hip` (rust/patches/0005-...) the task
//! instead awaits [`sign`]: the key and root go into the library's open window, the window closes at
//! `SSB_SIGN_MAX_JOBS` submissions or `SSB_SIGN_WINDOW_US` after its first, its distinct roots are
//! hashed once and the whole window is signed with ONE `ssb_sign_batch`; each task's oneshot completes
//! from the library's worker thread with exactly `SecretKey::sign`'s signature (the POP DST of
//! src/crypto/impls/blst.rs:11; the engine repository's tests/test_gpu_collector.py checks every
//! window's bytes against the C oracle's `sign` and the Ethereum consensus-spec `sign` vector).
//! If the engine is unavailable the reference's own CPU signing runs, with an error logged (a
//! duty's signature cannot be skipped: local_sign_and_store returns nothing).  Mirrors
//! `safestakeoperator_amd/collector.py` (`LocalSigner`); type-checked by inspection only (no cargo in
//! the engine's build image).
use bls::{Hash256, SecretKey, Signature};
use tokio::sync::oneshot;

use log::error;

use crate::crypto::impls::hip::engine;

/// Drop-in for `sk.sign(msg)` (dvfcore.rs:242): the same signature, awaited instead of computed on
/// the calling task.
pub async fn sign(sk: &SecretKey, msg: Hash256) -> Signature {
    let e = match engine() {
        Ok(e) => e,
        Err(err) => {
            error!("ssbls engine unavailable ({:?}): signing on the CPU", err);
            return sk.sign(msg);
        }
    };
    let (tx, rx) = oneshot::channel();
    if let Err(err) = e.sign_submit(sk, msg, tx) {
        error!("ssbls signing window refused a signature ({:?}): signing on the CPU", err);
        return sk.sign(msg);
    }
    match rx.await {
        Ok(Ok(sig)) => sig,
        other => {
            error!("ssbls signing window failed ({:?}): signing on the CPU", other.err());
            sk.sign(msg)
        }
    }
}
