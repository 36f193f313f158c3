"""GPU: every BASELINE.json config at its full per-GPU size, checked against INDEPENDENT
references -- the plain-C oracle (oracle/bls_c.c: 64-bit-limb restatement of the reference's scan,
exact per-share verify and Lagrange combine, tests/test_oracle_c.py pins it to the Python oracle and
the published vectors) and the construction truth of the inputs (which shares were signed over the
wrong root) -- not against the engine's own signer.

  C2  4,096 validators x 4, 3-of-4, 64 roots; all valid and 1% invalid: EVERY verdict, status and
      combined signature == the C oracle on the same bytes
  C3  65,536 validators 3-of-4: the 65,536 combined signatures verified on the device with the
      validators' master keys (a-8, ssb_verify_batch_cached_dev), plus swapped / out-of-range cases
  C4  1,048,576 shares at invalid rates 1e-4 and 1e-2: exact verdicts, statuses, combines
  C5  131,072 validators x 13, 10-of-13 (one GPU's slice of 1M): 64 roots and all-distinct roots
and the RFC 9380 Appendix K.2 hash_to_G2 vector (QUUX DST) on the device.
Reference test being generalised: tests/test_generic_threshold.rs:26-35 (combine == master
signature, both verify).
"""
import ctypes
import json
import os

import numpy as np
import pytest

import bench
from oracle import bls_c
from safestakeoperator_amd import DST, _lib

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
THREADS = 16


def _agg(engine, wl, V, t, n):
    offs = list(range(0, V * n + 1, n))
    return engine.threshold_aggregate_batch_raw([t] * V, offs, wl["sigs"], wl["pks"], wl["ids"], wl["job_root"],
                                                wl["roots"])


def _c_oracle(wl, jobs, t, n):
    """C oracle on the listed jobs (every share verified): (out96, status, err, verdicts)."""
    sig = b"".join(wl["sigs"][96 * n * v:96 * n * (v + 1)] for v in jobs)
    pk = b"".join(wl["pks"][48 * n * v:48 * n * (v + 1)] for v in jobs)
    ids = [i for v in jobs for i in wl["ids"][n * v:n * (v + 1)]]
    used = sorted({wl["job_root"][v] for v in jobs})       # hash only the roots the sample signs
    remap = {r: k for k, r in enumerate(used)}
    jr = [remap[wl["job_root"][v]] for v in jobs]
    off = list(range(0, len(jobs) * n + 1, n))
    return bls_c.threshold_batch(off, [t] * len(jobs), sig, pk, ids, jr, [wl["roots"][r] for r in used], THREADS,
                                 verify_all=True)


def _check_against_truth(wl, V, t, n, out, st, err, ver):
    valid = np.asarray(wl["valid"], dtype=np.uint8)
    assert (ver == valid).all(), np.nonzero(ver != valid)[0][:20]
    per_job = valid.reshape(V, n).sum(axis=1)
    assert ((st == 0) == (per_job >= t)).all()
    bad = np.nonzero(per_job < t)[0]
    assert (st[bad] == 4).all() and (err[bad, 0] == per_job[bad]).all() and (err[bad, 1] == t).all()


def test_rfc9380_k2_vector_on_gpu(engine):
    """RFC 9380 Appendix K.2 (BLS12381G2_XMD:SHA-256_SSWU_RO_, QUUX DST, msg = ""), published
    output point, through ssb_hash_to_g2_msgs."""
    v = json.load(open(os.path.join(GOLD, "known_answers.json")))["rfc9380_g2"][0]
    out = engine.hash_to_g2([v["msg"].encode()], dst=v["dst"].encode())[0].hex()
    assert [out[0:96], out[96:192], out[192:288], out[288:384]] == [v["P_x"][1], v["P_x"][0], v["P_y"][1], v["P_y"][0]]
    # the same message padded to a 32-byte root is a different input: a different point
    assert engine.hash_to_g2([bytes(32)], dst=v["dst"].encode())[0].hex() != out


@pytest.mark.parametrize("rate", [0.0, 0.01], ids=["valid", "invalid_1pct"])
def test_c2_full_batch_matches_c_oracle(engine, rate):
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=0, invalid_rate=rate)
    out, st, err, ver = _agg(engine, wl, V, t, n)
    o_out, o_st, o_err, o_ver = _c_oracle(wl, list(range(V)), t, n)
    assert (ver == o_ver[:V * n]).all(), np.nonzero(ver != o_ver[:V * n])[0][:20]
    assert (st == o_st).all()
    assert (err == o_err).all()
    ok = st == 0
    assert (out[ok] == o_out[ok]).all()
    _check_against_truth(wl, V, t, n, out, st, err, ver)
    assert rate == 0 or wl["n_bad"] > 100


@pytest.mark.parametrize("rate", [0.0, 0.01], ids=["valid", "invalid_1pct"])
def test_c2_one_stream_slots_match_c_oracle(engine, rate):
    """The throughput configuration bench.py runs: one-stream slots, every stage of a batch on its
    slot's stream (SSB_POST=slot: verdicts, the exact fallback -- group tests when the batch fails --
    and one combine from the verdicts, no speculative pass), several slots in turn.  Every verdict,
    status and combined signature == the C oracle on the same bytes."""
    lib = engine._lib
    assert lib.ssb_set_slot_streams(engine.handle, 1) == 0, lib.ssb_last_error(engine.handle)
    assert lib.ssb_set_pipeline_depth(engine.handle, 4) == 0, lib.ssb_last_error(engine.handle)
    try:
        V, t, n, R = 4096, 3, 4, 64
        wl = bench.make_workload(engine, V, t, n, R, rank=2, invalid_rate=rate)
        runs = [_agg(engine, wl, V, t, n) for _ in range(3)]          # three consecutive slots
        o_out, o_st, o_err, o_ver = _c_oracle(wl, list(range(V)), t, n)
        for out, st, err, ver in runs:
            assert (ver == o_ver[:V * n]).all(), np.nonzero(ver != o_ver[:V * n])[0][:20]
            assert (st == o_st).all() and (err == o_err).all()
            ok = st == 0
            assert (out[ok] == o_out[ok]).all()
            _check_against_truth(wl, V, t, n, out, st, err, ver)
        assert rate == 0 or wl["n_bad"] > 100
    finally:
        lib.ssb_set_pipeline_depth(engine.handle, 1)
        lib.ssb_set_slot_streams(engine.handle, 3)


def _oracle_signed(wl, threads=THREADS):
    """The workload's shares signed, and their keys derived, by the C oracle alone (bls_c.sign,
    bls_c.sk_to_pk: 64-bit-limb restatement, pinned by the Ethereum `sign` KAT and RFC 9380), from the
    same share secrets and signing roots -- inputs independent of the engine's own signer."""
    from concurrent.futures import ThreadPoolExecutor   # (ctypes calls release the GIL)
    sks = [k.to_bytes(32, "big") for k in wl["share_sk"]]
    with ThreadPoolExecutor(threads) as ex:
        sigs = list(ex.map(lambda a: bls_c.sign(a[0], wl["roots"][a[1]]), zip(sks, wl["sign_root"]), chunksize=256))
        pks = list(ex.map(bls_c.sk_to_pk, sks, chunksize=256))
    return sigs, pks


@pytest.mark.parametrize("pattern", ["valid", "invalid_1pct", "bad_operator"])
def test_c2_full_size_oracle_signed_inputs(engine, pattern):
    """Full C2 (4,096 x 3-of-4, 64 roots, 16,384 shares) on inputs the C ORACLE signed: the engine's
    batched signer and key derivation == the oracle's bytes for every share, and the engine's batch
    (every verdict, status, error and combined signature) == the oracle's scan on those bytes; every
    combined signature == bls_c.sign(master secret, root), i.e. the validator's own signature
    (tests/test_generic_threshold.rs:26-35 at full size)."""
    V, t, n, R = 4096, 3, 4, 64
    kw = {"invalid_rate": 0.01} if pattern == "invalid_1pct" else {"bad_operator": 2} if pattern == "bad_operator" else {}
    wl = bench.make_workload(engine, V, t, n, R, rank=5, **kw)
    sigs, pks = _oracle_signed(wl)
    assert sigs == wl["share_sigs"] and pks == wl["share_pks"]
    wl = dict(wl, sigs=b"".join(sigs), pks=b"".join(pks))
    out, st, err, ver = _agg(engine, wl, V, t, n)
    o_out, o_st, o_err, o_ver = _c_oracle(wl, list(range(V)), t, n)
    assert (ver == o_ver[:V * n]).all(), np.nonzero(ver != o_ver[:V * n])[0][:20]
    assert (st == o_st).all() and (err == o_err).all()
    ok = np.nonzero(st == 0)[0]
    assert (out[ok] == o_out[ok]).all()
    _check_against_truth(wl, V, t, n, out, st, err, ver)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(THREADS) as ex:
        master = list(ex.map(lambda v: bls_c.sign(int(wl["master"][v]).to_bytes(32, "big"), wl["roots"][wl["job_root"][v]]),
                             ok.tolist(), chunksize=128))
    assert [bytes(out[v]) for v in ok.tolist()] == master
    assert len(ok) == V if pattern != "invalid_1pct" else len(ok) > V - 100


def _verify_cached_dev(engine, cache_pk48, pk_index, sigs96, root_idx, roots, seed=None):
    import torch
    lib = engine._lib
    dev = torch.device("cuda", 0)
    u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    cache = np.frombuffer(b"".join(cache_pk48), dtype=np.uint8)
    assert lib.ssb_pk_cache_set(engine.handle, len(cache_pk48), cache.ctypes.data_as(_lib._u8p)) == 0
    n = len(sigs96)
    d_idx = torch.tensor(np.asarray(pk_index, dtype=np.uint32).view(np.int32), device=dev)
    d_sig, d_roots = u8(b"".join(sigs96)), u8(b"".join(roots))
    d_ri = torch.tensor(np.asarray(root_idx, dtype=np.uint32).view(np.int32), device=dev)
    d_ver = torch.zeros((n,), dtype=torch.uint8, device=dev)
    dst = (ctypes.c_uint8 * len(DST)).from_buffer_copy(DST)
    rc = lib.ssb_verify_batch_cached_dev(engine.handle, n, d_idx.data_ptr(), d_sig.data_ptr(), d_ri.data_ptr(), len(roots),
                                         d_roots.data_ptr(), ctypes.cast(dst, _lib._u8p), len(DST),
                                         int.from_bytes(os.urandom(8), "little"), d_ver.data_ptr(), None)
    assert rc == 0, lib.ssb_last_error(engine.handle)
    torch.cuda.synchronize()
    return d_ver.cpu().numpy()


def test_c3_final_verify_65536(engine):
    """a-8 at C3 size: combine 65,536 validators (3-of-4), then verify all 65,536 combined
    signatures on the device against the master keys (RLC across validators sharing a root, keys
    from the decoded-key cache).  Two swapped signatures, an out-of-range root and an out-of-range
    key index must be the only verdicts 0; a sample re-verified by the C oracle."""
    V, t, n, R = 65536, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=3)
    out, st, err, ver = _agg(engine, wl, V, t, n)
    assert (st == 0).all() and ver.all()
    mpk = engine.sk_to_pk_batch(wl["master"])
    comb = [out[v].tobytes() for v in range(V)]
    comb[100], comb[4000] = comb[4000], comb[100]          # swapped: both invalid
    ri = list(wl["job_root"])
    ri[777] = R + 9                                        # no such root
    pk_index = list(range(V))
    pk_index[31337] = V + 5                                # no such key
    got = _verify_cached_dev(engine, mpk, pk_index, comb, ri, wl["roots"])
    want = np.ones(V, dtype=np.uint8)
    want[[100, 4000, 777, 31337]] = 0
    assert (got == want).all(), np.nonzero(got != want)[0]
    for v in (0, 100, 4000, 65535):
        assert bls_c.verify(mpk[v], comb[v], wl["roots"][wl["job_root"][v]]) == bool(want[v])


@pytest.mark.parametrize("rate", [1e-4, 1e-2], ids=["1e-4", "1e-2"])
def test_c4_invalid_rates_full_size(engine, rate):
    """C4: 1,048,576 shares (262,144 validators x 4, 64 roots) in ONE batch at invalid rate 1e-4 /
    1e-2: every verdict and status exact (construction truth), and every job that lost a share
    combines to the same bytes as the C oracle (sampled: all such jobs up to 256)."""
    V, t, n, R = 262144, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=5, invalid_rate=rate)
    out, st, err, ver = _agg(engine, wl, V, t, n)
    _check_against_truth(wl, V, t, n, out, st, err, ver)
    valid = np.asarray(wl["valid"]).reshape(V, n)
    hit = np.nonzero(valid.sum(axis=1) < n)[0][:256].tolist() + [0, V - 1]
    o_out, o_st, o_err, o_ver = _c_oracle(wl, hit, t, n)
    assert (st[hit] == o_st).all()
    assert all(out[v].tobytes() == o_out[k].tobytes() for k, v in enumerate(hit) if st[v] == 0)
    assert wl["n_bad"] > (50 if rate < 1e-3 else 9000)


@pytest.mark.parametrize("distinct_roots", [False, True], ids=["64_roots", "all_distinct_roots"])
def test_c5_per_gpu_slice(engine, distinct_roots):
    """C5, one GPU's slice of 1M validators over 8: 131,072 validators x 13 shares, 10-of-13, with
    64 signing roots (one per committee) or every validator on its own root (hash_to_G2 of 131,072
    roots, one Miller pair per root).  All statuses Ok, every share verified, a sample of 128
    validators' combines == the C oracle's."""
    V, t, n = 131072, 10, 13
    R = V if distinct_roots else 64
    wl = bench.make_workload(engine, V, t, n, R, rank=7)
    out, st, err, ver = _agg(engine, wl, V, t, n)
    assert (st == 0).all() and ver.all()
    sample = list(range(0, V, V // 128))
    o_out, o_st, o_err, o_ver = _c_oracle(wl, sample, t, n)
    assert (o_st == 0).all() and o_ver[:len(sample) * n].all()
    assert all(out[v].tobytes() == o_out[k].tobytes() for k, v in enumerate(sample))


def test_twenty_slots_every_batch_in_fallback(engine):
    """20 one-stream slots in flight at once (the bench's configuration) with 1% invalid shares in
    EVERY batch, so every slot queue runs the exact group-test fallback -- the path whose larger
    kernels could grow a queue's scratch while the other queues run (round 2's
    HSA_STATUS_ERROR_OUT_OF_RESOURCES; every batch kernel now fits the queue primer, build guard).
    Twenty batches submitted through the asynchronous host path before any wait, each with its own
    invalid set: every verdict / status / combine == the construction truth, and the first and the
    last batch == the C oracle on the same bytes."""
    V, t, n, R, S = 512, 3, 4, 8, 20
    wl = bench.make_workload(engine, V, t, n, R, 31, invalid_rate=0.0)
    N = V * n
    wrong = engine.sign_batch([11 + i for i in range(N // 50)], [0] * (N // 50), [bytes([7]) * 32])
    rng = np.random.default_rng(77)
    batches = []
    for b in range(S):
        bad = sorted(rng.choice(N, size=N // 100, replace=False).tolist())
        sigs = bytearray(wl["sigs"])
        for k, i in enumerate(bad):
            sigs[96 * i:96 * (i + 1)] = wrong[(k + b) % len(wrong)]
        valid = np.ones(N, dtype=np.uint8)
        valid[bad] = 0
        batches.append((bytes(sigs), valid))
    lib = engine._lib
    assert lib.ssb_set_slot_streams(engine.handle, 1) == 0
    assert lib.ssb_set_pipeline_depth(engine.handle, S) == 0
    try:
        offs = list(range(0, N + 1, n))
        pend = [engine.submit_batch_raw([t] * V, offs, sg, wl["pks"], wl["ids"], wl["job_root"], wl["roots"])
                for sg, _ in batches]
        res = [p.wait() for p in pend]
    finally:
        lib.ssb_set_pipeline_depth(engine.handle, 1)
        lib.ssb_set_slot_streams(engine.handle, 3)
    msig = engine.sign_batch(wl["master"], wl["job_root"], wl["roots"])
    for (sg, valid), (out, st, err, ver) in zip(batches, res):
        assert (ver == valid).all()
        per_job = valid.reshape(V, n).sum(axis=1)
        assert ((st == 0) == (per_job >= t)).all()
        ok = np.nonzero(per_job >= t)[0]
        assert all(out[v].tobytes() == msig[v] for v in ok)
    for b in (0, S - 1):
        sg, _ = batches[b]
        o_out, o_st, o_err, o_ver = bls_c.threshold_batch(list(range(0, N + 1, n)), [t] * V, sg, wl["pks"], wl["ids"],
                                                          wl["job_root"], wl["roots"], THREADS, verify_all=True)
        out, st, err, ver = res[b]
        assert (ver == o_ver[:N]).all() and (st == o_st).all() and (err == o_err).all()
        assert (out[st == 0] == o_out[o_st == 0]).all()


def _cached_one_stream(engine, wl, V, t, n, slots=2, batches=None):
    """ssb_threshold_aggregate_batch_cached_dev on one-stream slots (bench.py's timed path: keys from
    the decoded-key cache, the fused launches), `batches` (default: one per slot) batches of the same
    inputs: [(out96, status, err, verdicts)]."""
    import ctypes
    import torch
    lib = engine._lib
    dev = torch.device("cuda", 0)
    N = V * n
    u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    cache = np.frombuffer(wl["pks"], dtype=np.uint8)
    assert lib.ssb_pk_cache_set(engine.handle, N, cache.ctypes.data_as(_lib._u8p)) == 0
    d_sig, d_roots = u8(wl["sigs"]), u8(b"".join(wl["roots"]))
    d_idx = torch.arange(0, N, dtype=torch.int32, device=dev)
    d_ids = torch.tensor(wl["ids"], dtype=torch.int64, device=dev)
    d_off = torch.arange(0, N + 1, n, dtype=torch.int32, device=dev)
    d_t = torch.full((V,), t, dtype=torch.int32, device=dev)
    d_jr = torch.tensor(wl["job_root"], dtype=torch.int32, device=dev)
    dst = (ctypes.c_uint8 * len(DST)).from_buffer_copy(DST)
    assert lib.ssb_set_slot_streams(engine.handle, 1) == 0, lib.ssb_last_error(engine.handle)
    assert lib.ssb_set_pipeline_depth(engine.handle, slots) == 0, lib.ssb_last_error(engine.handle)
    try:
        runs = []
        for k in range(batches or slots):
            out = torch.zeros((V, 96), dtype=torch.uint8, device=dev)
            st = torch.zeros((V,), dtype=torch.int32, device=dev)
            err = torch.zeros((V, 2), dtype=torch.int64, device=dev)
            ver = torch.zeros((N,), dtype=torch.uint8, device=dev)
            rc = lib.ssb_threshold_aggregate_batch_cached_dev(
                engine.handle, V, N, d_off.data_ptr(), d_t.data_ptr(), d_sig.data_ptr(), d_idx.data_ptr(), d_ids.data_ptr(),
                d_jr.data_ptr(), len(wl["roots"]), d_roots.data_ptr(), ctypes.cast(dst, _lib._u8p), len(DST), 0x5AFE + k,
                out.data_ptr(), st.data_ptr(), err.data_ptr(), ver.data_ptr(), None)
            assert rc == 0, lib.ssb_last_error(engine.handle)
            runs.append((out, st, err, ver))
        torch.cuda.synchronize()
        return [tuple(x.cpu().numpy() for x in r) for r in runs]
    finally:
        lib.ssb_set_pipeline_depth(engine.handle, 1)
        lib.ssb_set_slot_streams(engine.handle, 3)
        assert lib.ssb_pk_cache_set(engine.handle, 0, None) == 0


@pytest.mark.parametrize("g1", ["merged", "windowed"])
@pytest.mark.parametrize("rate", [0.0, 0.01, 0.95], ids=["valid", "invalid_1pct", "invalid_95pct"])
def test_c2_cached_one_stream_matches_c_oracle(engine, monkeypatch, g1, rate):
    """bench.py's timed path: one-stream slots, keys from the cache.  merged: the G1 sums read the
    cache's precomputed bases [2^(4w)] pk (one 16-bucket MSM per root, no Horner); windowed
    (SSB_NO_PKPOW=1): the per-window G1 MSM + Horner.  At 95% invalid shares most buckets are empty
    (infinity inputs to every reduction) and every batch runs the group-test fallback with its
    two-pair Miller loops.  Every verdict, status and combined signature == the C oracle on the
    same bytes."""
    if g1 == "windowed":
        monkeypatch.setenv("SSB_NO_PKPOW", "1")
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=3, invalid_rate=rate)
    runs = _cached_one_stream(engine, wl, V, t, n)
    o_out, o_st, o_err, o_ver = _c_oracle(wl, list(range(V)), t, n)
    for out, st, err, ver in runs:
        assert (ver == o_ver[:V * n]).all(), np.nonzero(ver != o_ver[:V * n])[0][:20]
        assert (st == o_st).all() and (err.astype(np.uint64) == o_err.astype(np.uint64)).all()
        ok = st == 0
        assert (out[ok] == o_out[ok]).all()
        _check_against_truth(wl, V, t, n, out, st, err, ver)


@pytest.mark.parametrize("rate", [0.0, 0.01, 0.95], ids=["valid", "invalid_1pct", "invalid_95pct"])
def test_c2_cached_depth1_latency_forms(engine, rate):
    """One batch in flight (ssb_set_pipeline_depth(1), one-stream slots, bench.py's batch_latency_ms):
    the MSM launches take their latency forms -- the G2 window sums as 8-lane programs in 128-lane
    blocks (k_msm_window2_lat), the cofactor clearing and the affine H(root) beside the bucket sums
    (k_msm_bucket2_clr).  At 95% invalid shares most buckets are empty, so the lane programs meet
    infinity and the windows are redone exactly in the same block.  Three batches on the one slot
    (the clearing's completion ticket must come back zeroed).  Every verdict, status and combined
    signature == the C oracle on the same bytes."""
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=5, invalid_rate=rate)
    runs = _cached_one_stream(engine, wl, V, t, n, slots=1, batches=3)
    o_out, o_st, o_err, o_ver = _c_oracle(wl, list(range(V)), t, n)
    for out, st, err, ver in runs:
        assert (ver == o_ver[:V * n]).all(), np.nonzero(ver != o_ver[:V * n])[0][:20]
        assert (st == o_st).all() and (err.astype(np.uint64) == o_err.astype(np.uint64)).all()
        ok = st == 0
        assert (out[ok] == o_out[ok]).all()
        _check_against_truth(wl, V, t, n, out, st, err, ver)


@pytest.mark.parametrize("count", [1, 3, 8], ids=["one", "three", "eight"])
def test_c2_cached_one_stream_few_invalid(engine, count):
    """A few invalid shares per C2 batch (bench.py --invalid-count): level 0 of the fallback checks
    each root against the batch check's own Miller value e(PK_r, H(r)) and a per-root bucket sum of
    k_i sig_i (k_fb_root); with at most FB_SINGLE_MAX (384) shares in failing roots -- one failing
    root of 256 -- they are checked one by one (k_fb_single), with more (three or eight roots)
    through the per-share products and the 16-ary levels.  Every verdict, status and combined
    signature == the C oracle on the same bytes."""
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=4, invalid_count=count)
    runs = _cached_one_stream(engine, wl, V, t, n)
    o_out, o_st, o_err, o_ver = _c_oracle(wl, list(range(V)), t, n)
    assert int((o_ver[:V * n] == 0).sum()) == count
    for out, st, err, ver in runs:
        assert (ver == o_ver[:V * n]).all(), np.nonzero(ver != o_ver[:V * n])[0][:20]
        assert (st == o_st).all() and (err.astype(np.uint64) == o_err.astype(np.uint64)).all()
        ok = st == 0
        assert (out[ok] == o_out[ok]).all()
        _check_against_truth(wl, V, t, n, out, st, err, ver)
