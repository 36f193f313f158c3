"""GPU: soundness of the random-linear-combination batch check against crafted shares.

The reference verifies every partial signature on its own (src/crypto/generic_threshold.rs:156), so a
share that is not sk_i * H(m) is always rejected.  The engine checks a whole batch with one
combination sum_i k_i sig_i; if the k_i were known to the senders, two of them could submit
    sig_a' = sig_a + [k_b] D,    sig_b' = sig_b - [k_a] D        (D any point of G2)
whose errors cancel in every sum that holds both (the batch, and the group tests of a failed
batch).  The engine draws a secret key per call (include/ssbls.h), so such a pair is caught:
both shares get verdict 0 and the jobs combine from their other shares, exactly as the reference.

The negative control runs the same crafted inputs on an engine switched to the deterministic
(test-only) key: there the pair passes, which proves the crafted pair is a real forgery against
known scalars -- and that the device derives exactly the scalars oracle/rlc.py restates.
"""
import hashlib

import numpy as np
import pytest

from oracle import bls12_381 as B
from oracle import rlc

from test_gpu_parity import _gen_committees

pytestmark = pytest.mark.gpu

SEED = 0x5AFE57A4E          # the round-1 default seed (public)


def _forge(sigs, a, b, ka, kb, tag=b"delta"):
    """sig_a + [k_b] D, sig_b - [k_a] D"""
    D = B.hash_to_g2(hashlib.sha256(tag).digest())
    out = list(sigs)
    sa, sb = B.g2_decompress(sigs[a]), B.g2_decompress(sigs[b])
    out[a] = B.g2_compress(B.g2_add(sa, B.g2_mul(D, kb)))
    out[b] = B.g2_compress(B.g2_add(sb, B.g2_neg(B.g2_mul(D, ka))))
    return out


def _run(engine, t, V, n, sigs, pks, ids, jr, roots, seed):
    offs = list(range(0, V * n + 1, n))
    return engine.threshold_aggregate_batch_raw([t] * V, offs, b"".join(sigs), b"".join(pks), ids, jr, roots, seed=seed)


@pytest.fixture
def committees(engine):
    V, t, n = 64, 3, 4
    roots, master, sigs, pks, ids, jr, msig = _gen_committees(engine, V, t, n, 4, seed=41)
    return V, t, n, roots, master, list(sigs), pks, ids, jr, msig


def _expect_exact(V, t, n, ver, st, err, out, msig, bad):
    expect = np.ones(V * n, dtype=np.uint8)
    expect[bad] = 0
    assert (ver == expect).all(), np.nonzero(ver != expect)[0]
    for v in range(V):
        valid = int(expect[v * n:(v + 1) * n].sum())
        if valid >= t:
            assert st[v] == 0 and out[v].tobytes() == msig[v], v
        else:
            assert st[v] == 4 and list(err[v]) == [valid, t], v


def test_forged_pair_passes_only_with_known_scalars(engine, committees):
    """Negative control + device pin: with the deterministic key the pair built from
    oracle/rlc.py's scalars passes the batch (so the device scalars ARE those), and the
    combine of validator 0 comes out wrong; the default engine rejects the same bytes."""
    V, t, n, roots, master, sigs, pks, ids, jr, msig = committees
    a, b = 0, 5 * n + 1                               # validator 0 share 0, validator 5 share 1
    ks = rlc.deterministic_scalars(SEED, V * n)
    forged = _forge(sigs, a, b, ks[a], ks[b])
    assert not B.verify(pks[a], forged[a], roots[jr[0]]) and not B.verify(pks[b], forged[b], roots[jr[5]])
    try:
        engine.set_rlc_deterministic(True)
        out, st, err, ver = _run(engine, t, V, n, forged, pks, ids, jr, roots, SEED)
    finally:
        engine.set_rlc_deterministic(False)
    assert ver.all(), "the crafted pair should cancel under known scalars"
    assert out[0].tobytes() != msig[0]
    out, st, err, ver = _run(engine, t, V, n, forged, pks, ids, jr, roots, SEED)
    _expect_exact(V, t, n, ver, st, err, out, msig, [a, b])


@pytest.mark.parametrize("scalars", ["round1_default_seed", "deterministic_same_seed"])
def test_forged_pair_across_validators_rejected(engine, committees, scalars):
    """The pair in two different validators' jobs, built from the scalars an attacker could know
    (round 1's public splitmix scalars for the old default seed, or the deterministic key of the
    seed the caller passes): both shares verdict 0, both jobs combine from their other shares."""
    V, t, n, roots, master, sigs, pks, ids, jr, msig = committees
    a, b = 2 * n + 2, 9 * n + 0
    ks = rlc.round1_scalars(SEED, V * n) if scalars.startswith("round1") else rlc.deterministic_scalars(SEED, V * n)
    forged = _forge(sigs, a, b, ks[a], ks[b])
    out, st, err, ver = _run(engine, t, V, n, forged, pks, ids, jr, roots, SEED)
    _expect_exact(V, t, n, ver, st, err, out, msig, [a, b])
    # and through the reference-shaped API, one job at a time (oracle agrees)
    from safestakeoperator_amd import InsufficientValidSignatures, ThresholdSignature
    ts = ThresholdSignature(t, engine)
    v = a // n
    got = ts.threshold_aggregate(forged[v * n:(v + 1) * n], pks[v * n:(v + 1) * n], ids[v * n:(v + 1) * n], roots[jr[v]])
    st_o, pl_o = B.threshold_aggregate(t, forged[v * n:(v + 1) * n], pks[v * n:(v + 1) * n], ids[v * n:(v + 1) * n],
                                       roots[jr[v]])
    assert st_o == B.OK and pl_o == got == msig[v]


def test_forged_pair_in_one_job_insufficient(engine, committees):
    """Both crafted shares in ONE 3-of-4 job: the reference finds 2 valid shares ->
    InsufficientValidSignatures{got: 2, expected: 3}; so does the engine."""
    V, t, n, roots, master, sigs, pks, ids, jr, msig = committees
    a, b = 7 * n + 1, 7 * n + 3
    ks = rlc.deterministic_scalars(SEED, V * n)
    forged = _forge(sigs, a, b, ks[a], ks[b])
    out, st, err, ver = _run(engine, t, V, n, forged, pks, ids, jr, roots, SEED)
    _expect_exact(V, t, n, ver, st, err, out, msig, [a, b])
    assert st[7] == 4 and list(err[7]) == [2, 3]
    st_o, pl_o = B.threshold_aggregate(t, forged[7 * n:8 * n], pks[7 * n:8 * n], ids[7 * n:8 * n], roots[jr[7]])
    assert st_o == B.INSUFFICIENT_VALID_SIGNATURES and list(pl_o) == [2, 3]


@pytest.mark.parametrize("fallback", ["bisect", "share"])
def test_forged_pair_in_failed_batch_group_tests(engine, committees, fallback, monkeypatch):
    """A genuinely invalid share in the same root group makes the batch fail, so the verdicts come
    from the group tests of the fallback tree, which reuse the batch's scalars: the crafted pair
    (same root as the invalid share) is still caught, every verdict exact."""
    monkeypatch.setenv("SSB_FALLBACK", fallback)
    V, t, n, roots, master, sigs, pks, ids, jr, msig = committees
    r = jr[3]
    same_root = [v for v in range(V) if jr[v] == r]
    a, b, c = same_root[0] * n + 1, same_root[1] * n + 2, same_root[2] * n + 0
    ks = rlc.deterministic_scalars(SEED, V * n)
    forged = _forge(sigs, a, b, ks[a], ks[b])
    forged[c] = engine.sign_batch([12345], [0], [hashlib.sha256(b"elsewhere").digest()])[0]
    out, st, err, ver = _run(engine, t, V, n, forged, pks, ids, jr, roots, SEED)
    _expect_exact(V, t, n, ver, st, err, out, msig, [a, b, c])


def test_forged_pair_verify_batch(engine, committees):
    """ssb_verify_batch (a-2 / a-8 entry point) on the crafted pair: verdicts equal the
    per-share verify of the oracle."""
    V, t, n, roots, master, sigs, pks, ids, jr, msig = committees
    N = V * n
    ri = [jr[s // n] for s in range(N)]
    a, b = 11, 200
    ks = rlc.deterministic_scalars(SEED, N)
    forged = _forge(sigs, a, b, ks[a], ks[b])
    got = engine.verify_batch(pks, forged, ri, roots, seed=SEED)
    want = np.ones(N, dtype=np.uint8)
    want[[a, b]] = 0
    assert (got == want).all()
    assert not B.verify(pks[a], forged[a], roots[ri[a]])
