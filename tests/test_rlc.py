"""CPU: the RLC scalar derivation restated in oracle/rlc.py is the ChaCha block function of
RFC 8439 (pinned by its published test vector), scalars are odd and non-repeating, and the host
API never passes a fixed public seed; malformed jobs fail alone (batch and collector)."""
import secrets

import pytest

from oracle import rlc


def test_chacha20_block_rfc8439_vector():
    """RFC 8439 §2.3.2: key 00..1f, counter 1, nonce 00000009 0000004a 00000000 (20 rounds)."""
    key = [int.from_bytes(bytes(range(4 * k, 4 * k + 4)), "little") for k in range(8)]
    nonce = [int.from_bytes(bytes.fromhex(h), "little") for h in ("00000009", "0000004a", "00000000")]
    st = list(rlc.SIGMA) + key + [1] + nonce
    out = b"".join(w.to_bytes(4, "little") for w in rlc.chacha_block(st, 20))
    assert out.hex() == ("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                         "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def test_scalars_odd_distinct():
    key = [secrets.randbits(32) for _ in range(8)]
    ks = [rlc.rlc_scalar_odd(key, i) for i in range(4096)]
    assert all(k & 1 for k in ks) and len(set(ks)) == len(ks)
    assert rlc.deterministic_scalars(7, 4) == rlc.deterministic_scalars(7, 4)
    assert rlc.deterministic_scalars(7, 4) != rlc.deterministic_scalars(8, 4)


def test_host_api_seeds_are_random():
    from safestakeoperator_amd import threshold
    a = {threshold._rlc_seed(None) for _ in range(64)}
    assert len(a) == 64
    assert threshold._rlc_seed(5) == 5
    import inspect
    for fn in (threshold.Engine.verify_batch, threshold.Engine.threshold_aggregate_batch_raw,
               threshold.ThresholdSignature.threshold_aggregate_batch):
        assert inspect.signature(fn).parameters["seed"].default is None, fn


def test_malformed_jobs_fail_alone_in_a_batch():
    """Every job malformed: per-job errors, and no engine is needed (nothing reaches the device)."""
    from safestakeoperator_amd import DifferentLength, ThresholdJob, ThresholdSignature
    ts = ThresholdSignature(3, engine=object())          # never touched
    jobs = [ThresholdJob([b"\0" * 96] * 3, [b"\0" * 48] * 3, [1, 2, 3], b"short"),
            ThresholdJob([b"\0" * 95] * 3, [b"\0" * 48] * 3, [1, 2, 3], b"\0" * 32),
            ThresholdJob([b"\0" * 96] * 3, [b"\0" * 48] * 2, [1, 2, 3], b"\0" * 32),
            ThresholdJob([b"\0" * 96] * 3, [b"\0" * 48] * 3, [1, 2, -1], b"\0" * 32)]
    res = ts.threshold_aggregate_batch(jobs)
    assert isinstance(res[0], ValueError) and isinstance(res[1], ValueError) and isinstance(res[3], ValueError)
    assert res[2] == DifferentLength(3, 2)
    with pytest.raises(ValueError):
        ts.threshold_aggregate(*jobs[0].__dict__.values())
