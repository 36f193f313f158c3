//! tests/test_hip_threshold.rs -- the reference's tests/test_generic_threshold.rs, through the
//! batched entry point and the MI355X backend.  On a host with an MI355X:
//!     SSBLS_DIR=/path/to/engine cargo test --features hip --test test_hip_threshold
#![cfg(feature = "hip")]
use bls::{PublicKey, Signature};
use dvf::crypto::generic_threshold::ThresholdJob;
use dvf::crypto::ThresholdSignature;
use dvf::utils::error::DvfError;
use ethereum_hashing::{Context, Sha256Context};
use types::Hash256;

fn root(msg: &str) -> Hash256 {
    let mut context = Context::new();
    context.update(msg.as_bytes());
    Hash256::from_slice(&context.finalize())
}

#[test]
fn test_hip_threshold_batch() {
    let (t, n) = (5, 10);
    let mut m_threshold = ThresholdSignature::new(t);
    let ids = (1..n + 1).map(|k| k as u64).collect::<Vec<u64>>();
    let (kp, kps) = m_threshold.key_gen(&ids).unwrap();
    let pks: Vec<&PublicKey> = ids.iter().map(|id| &kps[id].pk).collect();
    let messages = [root("hello world"), root("second root")];
    let sigs: Vec<Vec<Signature>> = messages.iter().map(|m| ids.iter().map(|id| kps[id].sk.sign(*m)).collect()).collect();
    let refs: Vec<Vec<&Signature>> = sigs.iter().map(|v| v.iter().collect()).collect();
    // an invalid share first (signed over the other root): the scan moves past it
    let mut mixed = refs[0].clone();
    mixed[0] = refs[1][0];
    let zero_ids: Vec<u64> = ids.iter().map(|i| if *i == 2 { 0 } else { *i }).collect();
    let jobs = vec![
        ThresholdJob { sigs: &refs[0], pks: &pks, ids: &ids, msg: messages[0] },
        ThresholdJob { sigs: &refs[1], pks: &pks, ids: &ids, msg: messages[1] },
        ThresholdJob { sigs: &mixed, pks: &pks, ids: &ids, msg: messages[0] },
        ThresholdJob { sigs: &refs[0][..t - 1], pks: &pks[..t - 1], ids: &ids[..t - 1], msg: messages[0] },
        ThresholdJob { sigs: &refs[0], pks: &pks, ids: &zero_ids, msg: messages[0] },
        ThresholdJob { sigs: &refs[0], pks: &pks[..n - 1], ids: &ids, msg: messages[0] },
    ];
    let got = m_threshold.threshold_aggregate_batch(&jobs);
    // every job exactly as the per-job call (lighthouse verify loop + unsafe_aggregate)
    for (j, job) in jobs.iter().enumerate() {
        let want = m_threshold.threshold_aggregate(job.sigs, job.pks, job.ids, job.msg);
        assert_eq!(got[j], want, "job {}", j);
    }
    // tests/test_generic_threshold.rs:28-35: the combine equals the master key's signature
    for (k, m) in messages.iter().enumerate() {
        let sig = kp.sk.sign(*m);
        assert!(got[k].as_ref().unwrap().verify(&kp.pk, *m));
        assert_eq!(got[k].as_ref().unwrap(), &sig);
    }
    assert_eq!(got[2].as_ref().unwrap(), &kp.sk.sign(messages[0]));
    assert_eq!(got[3], Err(DvfError::InsufficientSignatures { got: t - 1, expected: t }));
    assert_eq!(got[4], Err(DvfError::InvalidOperatorId { id: 0 }));
    assert_eq!(got[5], Err(DvfError::DifferentLength { x: n, y: n - 1 }));
}
