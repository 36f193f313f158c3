"""GPU: the per-slot collector (include/ssbls.h "Per-slot collector", csrc/ssb_collector.hip) -- the
native batched caller SafeStake's per-duty tasks use instead of one threshold_aggregate call each
(HotstuffOperatorCommittee::sign, src/validation/impls/hotstuff.rs:141-169) -- and the incremental
key registration it runs on (ssb_pk_cache_add, committees registered as they are built).

Full C2 batches (4,096 validators x 4, 3-of-4, 64 roots) pushed job by job from native submitter
threads (bench_tools/collbench.cpp, the driver of bench.py's value_collector), several windows in
flight: every job's status, error fields, share verdicts and combined signature == the plain-C oracle
(oracle/bls_c.c) on the same bytes."""
import ctypes
import json
import os
import threading

import numpy as np
import pytest

import bench
from oracle import bls_c
from safestakeoperator_amd import Engine
from safestakeoperator_amd.collector import NativeCollector, SlotCollector, collbench_run
from safestakeoperator_amd.threshold import ThresholdJob, _error_from

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


def _oracle(wl, V, t, n):
    off = list(range(0, V * n + 1, n))
    return bls_c.threshold_batch(off, [t] * V, wl["sigs"], wl["pks"], wl["ids"], wl["job_root"], wl["roots"], 16,
                                 verify_all=True)


def _check(res, V, n, o_out, o_st, o_err, o_ver):
    k = np.arange(len(res))
    v = k % V
    assert (res["done"] == 1).all() and (res["rc"] == 0).all()
    assert (res["status"] == o_st[v]).all(), np.nonzero(res["status"] != o_st[v])[0][:10]
    assert (res["err"].astype(np.uint64) == o_err[v].astype(np.uint64)).all()
    ok = res["status"] == 0
    assert (res["sig96"][ok] == o_out[v[ok]]).all()
    # share verdicts (bit i of the job's word)
    ver = o_ver[:V * n].reshape(V, n).astype(np.uint64)
    want = (ver << np.arange(n, dtype=np.uint64)).sum(axis=1)
    assert (res["verdicts"] == want[v]).all()
    assert (res["n_shares"] == n).all()


@pytest.mark.parametrize("rate", [0.0, 0.01], ids=["valid", "invalid_1pct"])
def test_collector_full_c2_matches_c_oracle(eng, rate):
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(eng, V, t, n, R, rank=11, invalid_rate=rate)
    o_out, o_st, o_err, o_ver = _oracle(wl, V, t, n)
    col = NativeCollector(eng, max_jobs=4096, window_s=0.002, in_flight=4)
    try:
        rows = col.rows(wl["share_pks"])
        assert len(set(rows.tolist())) == V * n   # distinct keys -> distinct rows
        # three full windows of 8 interleaved submitters, then a partial one closed by its timer
        sec, res = collbench_run(col, wl, V, n, t, rows, 3 * V + 1000, threads=8)
        _check(res, V, n, o_out, o_st, o_err, o_ver)
        w, j, s = col.stats()
        assert j == 3 * V + 1000 and s == j * n and w >= 4
    finally:
        col.close()


def test_pk_cache_add_stable_rows(eng):
    """ssb_pk_cache_add: known keys keep their rows (also across a _set), new ones are appended, a
    key repeated inside one call gets one row; capacity growth keeps the earlier rows valid (a batch
    through rows registered before and after the growth matches the oracle)."""
    V, t, n, R = 400, 3, 4, 8
    wl = bench.make_workload(eng, V, t, n, R, rank=12)
    pks = wl["share_pks"]
    eng.pk_cache_set(pks[:10])
    r0 = eng.pk_cache_add(pks[5:15] + pks[5:7])
    assert r0.tolist() == list(range(5, 10)) + list(range(10, 15)) + [5, 6]
    r1 = eng.pk_cache_add(pks)               # grows past the first 1,024-row capacity
    assert r1.tolist() == list(range(len(pks)))
    col = NativeCollector(eng, max_jobs=256, window_s=0.001, in_flight=2)
    try:
        rows = col.rows(pks)
        assert rows.tolist() == list(range(len(pks)))
        o_out, o_st, o_err, o_ver = _oracle(wl, V, t, n)
        _, res = collbench_run(col, wl, V, n, t, rows, 2 * V, threads=4)
        _check(res, V, n, o_out, o_st, o_err, o_ver)
    finally:
        col.close()


def _cases():
    with open(os.path.join(GOLD, "threshold_cases.json")) as f:
        return json.load(f)["cases"]


def test_slot_collector_native_golden_concurrent(eng):
    """SlotCollector on the native collector: every golden case (errors in the reference's order,
    duplicate ids, undecodable / infinity / non-subgroup shares, t = 1, 5-of-10, 10-of-13) from
    16 concurrent Python submitters, each future == the golden expectation; a DifferentLength job
    fails alone."""
    cases = _cases()
    out = {}
    with SlotCollector(eng, max_jobs=64, window_s=0.003, in_flight=3) as col:
        def task(k):
            c = cases[k % len(cases)]
            j = ThresholdJob([bytes.fromhex(s) for s in c["sigs"]], [bytes.fromhex(p) for p in c["pks"]], c["ids"],
                             bytes.fromhex(c["root"]))
            try:
                out[k] = col.submit(c["t"], j).result(60)
            except Exception as e:  # noqa: BLE001 (DvfError is the expected outcome of some cases)
                out[k] = e
        th = [threading.Thread(target=task, args=(k,)) for k in range(16 * len(cases))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        c0 = cases[0]
        bad = col.submit(c0["t"], ThresholdJob([bytes.fromhex(s) for s in c0["sigs"]][:3],
                                               [bytes.fromhex(p) for p in c0["pks"]], c0["ids"], bytes.fromhex(c0["root"])))
        with pytest.raises(Exception) as ei:
            bad.result(10)
        assert type(ei.value).__name__ == "DifferentLength"
    for k, r in out.items():
        c = cases[k % len(cases)]
        if c["expected_status"] == 0:
            assert r == bytes.fromhex(c["master_sig"]), c["name"]
        else:
            pl = c["expected_payload"]
            assert r == _error_from(c["expected_status"], pl[0], pl[1] if len(pl) > 1 else 0), c["name"]
    assert len(out) == 16 * len(cases)


def _wire_case(eng):
    """A 3-of-4 batch whose shares travel as wire records (bincode(bls::Signature)), with records that
    do not deserialize -- the reference drops such a share before threshold_aggregate
    (RemoteOperator::sign, src/validation/operator.rs:108-131, and `.flatten()`, hotstuff.rs:150-155).
    Returns the workload, the records, their per-share lengths, and the expected (present) shares."""
    from safestakeoperator_amd.collector import wire_records
    V, t, n, R = 1024, 3, 4, 16
    wl = bench.make_workload(eng, V, t, n, R, rank=31)
    wl2 = bench.make_workload(eng, V, t, n, R, rank=31, invalid_rate=1.0)   # every share over the next root
    rec = bytearray(wire_records(wl["sigs"]))
    lens = [202] * (V * n)
    absent = set()

    def put(s, b):
        rec[202 * s:202 * s + 202] = b

    def r(s):
        return bytes(rec[202 * s:202 * s + 202])
    put(3 * n + 1, (195).to_bytes(8, "little") + r(3 * n + 1)[8:]); absent.add(3 * n + 1)          # length field
    put(5 * n + 0, r(5 * n)[:8] + b"1x" + r(5 * n)[10:]); absent.add(5 * n)                          # prefix
    put(5 * n + 2, r(5 * n + 2)[:40] + b"zz" + r(5 * n + 2)[42:]); absent.add(5 * n + 2)             # hex digit
    put(7 * n + 1, r(7 * n + 1)[:10] + b"9f" + b"ff" * 47 + r(7 * n + 1)[106:]); absent.add(7 * n + 1)   # x.c1 >= p
    put(9 * n + 0, r(9 * n)[:10] + b"00" + r(9 * n)[12:]); absent.add(9 * n)                         # no compression flag
    sigs = bytearray(wl["sigs"])
    sigs[96 * (9 * n + 1):96 * (9 * n + 2)] = wl2["sigs"][96 * (9 * n + 1):96 * (9 * n + 2)]       # present, invalid
    put(9 * n + 1, wire_records(bytes(sigs[96 * (9 * n + 1):96 * (9 * n + 2)])))
    lens[11 * n + 3] = 150; absent.add(11 * n + 3)                                                  # truncated record
    lens[17 * n + 2] = 260   # trailing bytes after the record: bincode::deserialize ignores them (present)
    inf = b"\xc0" + b"\x00" * 95
    sigs[96 * (13 * n + 2):96 * (13 * n + 3)] = inf                                                 # infinity: present, invalid
    put(13 * n + 2, wire_records(inf))
    up = r(15 * n + 1)
    put(15 * n + 1, up[:10] + up[10:].upper())                                                      # upper-case hex parses
    for k in range(40, 1024, 97):                                                                   # scattered drops
        s = k * n + (k % n)
        put(s, (0).to_bytes(8, "little") + r(s)[8:]); absent.add(s)
    wl["sigs"] = bytes(sigs)
    # the reference's view: each job's PRESENT shares, in order
    off, sg, pk, ids = [0], b"", b"", []
    for v in range(V):
        for i in range(n):
            s = v * n + i
            if s in absent:
                continue
            sg += wl["sigs"][96 * s:96 * s + 96]; pk += wl["pks"][48 * s:48 * s + 48]; ids.append(wl["ids"][s])
        off.append(len(ids))
    o_out, o_st, o_err, o_ver = bls_c.threshold_batch(off, [t] * V, sg, pk, ids, wl["job_root"], wl["roots"], 16,
                                                      verify_all=True)
    ver = np.zeros(V * n, dtype=np.uint8)
    keep = [s for s in range(V * n) if s not in absent]
    ver[keep] = o_ver[:len(keep)]
    assert o_st[5] == 2 and tuple(o_err[5]) == (2, 3)          # InsufficientSignatures{got: 2, expected: 3}
    assert o_st[9] == 4 and tuple(o_err[9]) == (2, 3)          # InsufficientValidSignatures{got: 2, expected: 3}
    return wl, bytes(rec), lens, absent, (o_out, o_st, o_err, ver), (V, t, n, R)


def test_wire_collector_drops_undecodable_shares(eng):
    """A wire collector (ssb_collector_create2(.., SSB_COLLECTOR_WIRE)): jobs submitted as the records
    operators send (ssb_collector_submit_wire), decoded on the device.  A record that does not
    deserialize -- bad length field, prefix, hex digit, x >= p, no compression flag, truncated -- makes
    its share ABSENT: two absent shares of a 3-of-4 job give the reference's InsufficientSignatures
    {got: 2, expected: 3}, not an invalid-share error; the absent bits say which.  Every status, error
    field, verdict and combined signature == the C oracle on each job's present shares."""
    from safestakeoperator_amd import _lib
    wl, rec, lens, absent, (o_out, o_st, o_err, o_ver), (V, t, n, R) = _wire_case(eng)
    col = NativeCollector(eng, max_jobs=256, window_s=0.002, in_flight=3, wire=True)
    try:
        rows = col.rows(wl["share_pks"])
        res = [_lib.JobResult() for _ in range(V)]
        keep = []
        for v in range(V):
            recs = [rec[202 * (v * n + i):202 * (v * n + i) + min(lens[v * n + i], 202)] +
                    (b"\x07junk" * 12)[:max(0, lens[v * n + i] - 202)] for i in range(n)]
            r_ = np.ascontiguousarray(rows[v * n:(v + 1) * n], dtype=np.uint32)
            ids = np.asarray(wl["ids"][v * n:(v + 1) * n], dtype=np.uint64)
            keep.append((r_, ids))
            col.submit_wire(t, recs, r_, ids, wl["roots"][wl["job_root"][v]], res[v])
        col.flush()
    finally:
        col.close()
    for v in range(V):
        r = res[v]
        assert r.done == 1 and r.rc == 0
        assert r.status == o_st[v] and (r.err[0], r.err[1]) == (o_err[v][0], o_err[v][1]), v
        if r.status == 0:
            assert bytes(r.sig96) == o_out[v].tobytes(), v
        want_abs = sum(1 << i for i in range(n) if v * n + i in absent)
        assert r.absent == want_abs, v
        want_ver = sum(int(o_ver[v * n + i]) << i for i in range(n))
        assert r.verdicts == want_ver, v


def test_wire_aggregate_entry_point(eng):
    """ssb_threshold_aggregate_batch_wire_cached_dev (one batch, device buffers): the same records,
    statuses per share (1 length, 2 prefix, 3 hex, 4 not a point), the same results as the oracle."""
    import torch
    from safestakeoperator_amd import DST, _lib
    wl, rec, lens, absent, (o_out, o_st, o_err, o_ver), (V, t, n, R) = _wire_case(eng)
    rec = bytearray(rec)
    for s, l in enumerate(lens):
        if l < 202:
            rec[202 * s:202 * s + 8] = (0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")   # what the collector stores
    N = V * n
    eng.pk_cache_set(wl["share_pks"])
    dev = torch.device("cuda", 0)
    d = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_rec, d_roots = d(bytes(rec)), d(b"".join(wl["roots"]))
    d_off = torch.arange(0, N + 1, n, dtype=torch.int32, device=dev)
    d_t = torch.full((V,), t, dtype=torch.int32, device=dev)
    d_pk = torch.arange(0, N, dtype=torch.int32, device=dev)
    d_ids = torch.tensor(wl["ids"], dtype=torch.int64, device=dev)
    d_jr = torch.tensor(wl["job_root"], dtype=torch.int32, device=dev)
    out = torch.zeros((V, 96), dtype=torch.uint8, device=dev)
    st = torch.zeros((V,), dtype=torch.int32, device=dev)
    err = torch.zeros((V, 2), dtype=torch.int64, device=dev)
    ver = torch.zeros((N,), dtype=torch.uint8, device=dev)
    wst = torch.full((N,), -1, dtype=torch.int32, device=dev)
    lib = eng._lib
    dst = (ctypes.c_uint8 * len(DST)).from_buffer_copy(DST)
    rc = lib.ssb_threshold_aggregate_batch_wire_cached_dev(
        eng.handle, V, N, d_off.data_ptr(), d_t.data_ptr(), d_rec.data_ptr(), 202, d_pk.data_ptr(), d_ids.data_ptr(),
        d_jr.data_ptr(), R, d_roots.data_ptr(), ctypes.cast(dst, _lib._u8p), len(DST), 7, out.data_ptr(), st.data_ptr(),
        err.data_ptr(), ver.data_ptr(), wst.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    assert rc == 0, lib.ssb_last_error(eng.handle)
    torch.cuda.synchronize(dev)
    st, err, out, ver, wst = st.cpu().numpy(), err.cpu().numpy(), out.cpu().numpy(), ver.cpu().numpy(), wst.cpu().numpy()
    assert (st == o_st).all() and (err.astype(np.uint64) == o_err.astype(np.uint64)).all()
    ok = st == 0
    assert (out[ok] == o_out[ok]).all()
    assert (ver == o_ver).all()
    assert sorted(np.nonzero(wst)[0].tolist()) == sorted(absent)
    assert wst[3 * n + 1] == 1 and wst[5 * n] == 2 and wst[5 * n + 2] == 3 and wst[7 * n + 1] == 4 and wst[9 * n] == 4
    assert wst[11 * n + 3] == 1 and wst[13 * n + 2] == 0 and wst[15 * n + 1] == 0


def test_collector_owns_slot_configuration(eng):
    """while a collector is attached its slots are its own -- ssb_set_pipeline_depth /
    ssb_set_slot_streams return SSB_EINVAL (a depth below in_flight used to leave its worker a null
    slot stream), a second collector must use the same in_flight; after ssb_collector_destroy the
    context is reconfigurable again."""
    lib = eng._lib
    col = NativeCollector(eng, max_jobs=64, window_s=0.001, in_flight=2)
    try:
        assert lib.ssb_set_pipeline_depth(eng.handle, 1) == -1
        assert b"collector is attached" in lib.ssb_last_error(eng.handle)
        assert lib.ssb_set_slot_streams(eng.handle, 3) == -1
        with pytest.raises(RuntimeError):
            NativeCollector(eng, max_jobs=64, window_s=0.001, in_flight=3)
        col2 = NativeCollector(eng, max_jobs=64, window_s=0.001, in_flight=2)
        col2.close()
        assert lib.ssb_set_pipeline_depth(eng.handle, 3) == -1   # still attached: col
        # the collector still works after the refused calls (every golden-free job of a small batch)
        V, t, n, R = 64, 3, 4, 4
        wl = bench.make_workload(eng, V, t, n, R, rank=41)
        rows = col.rows(wl["share_pks"])
        _, res = collbench_run(col, wl, V, n, t, rows, V, threads=2)
        _check(res, V, n, *_oracle(wl, V, t, n))
    finally:
        col.close()
    assert lib.ssb_set_pipeline_depth(eng.handle, 3) == 0 and lib.ssb_set_slot_streams(eng.handle, 1) == 0
    assert lib.ssb_set_pipeline_depth(eng.handle, 1) == 0


def test_collector_beside_direct_calls(eng):
    """ONE engine serves a live collector and direct calls from another thread at the same
    time -- native submitters push 4 x 1,024 C2-shaped jobs while a Python thread runs whole
    threshold_aggregate_batch calls (host buffers: ssb_batch_wait polls outside the context lock),
    unsafe_aggregate (a synchronous entry point: waits outside the lock, on an idle slot when there is
    one) and registers new keys (ssb_pk_cache_add).  Every collector job == the C oracle, every direct
    result == the oracle / the master signature, and new keys get fresh rows."""
    from safestakeoperator_amd import ThresholdSignature
    V, t, n, R = 1024, 3, 4, 16
    wl = bench.make_workload(eng, V, t, n, R, rank=43, invalid_rate=0.01)
    o = _oracle(wl, V, t, n)
    wd = bench.make_workload(eng, 48, t, n, 4, rank=44)
    od_out, od_st, od_err, _ = _oracle(wd, 48, t, n)
    extra = bench.make_workload(eng, 64, t, n, 2, rank=45)["share_pks"]
    col = NativeCollector(eng, max_jobs=256, window_s=0.001, in_flight=4)
    errors, direct = [], {"batch": 0, "unsafe": 0}
    stop = threading.Event()

    def direct_calls():
        try:
            ts = ThresholdSignature(t, eng)
            k = 0
            while not stop.is_set() or k < 3:
                jobs = [ThresholdJob([wd["sigs"][96 * (v * n + i):96 * (v * n + i + 1)] for i in range(n)],
                                     wd["share_pks"][v * n:(v + 1) * n], wd["ids"][v * n:(v + 1) * n],
                                     wd["roots"][wd["job_root"][v]]) for v in range(48)]
                out = ts.threshold_aggregate_batch(jobs)
                for v in range(48):
                    assert od_st[v] == 0 and out[v] == od_out[v].tobytes(), ("batch", v)
                direct["batch"] += 1
                v = k % 48
                u = ts.unsafe_aggregate([wd["sigs"][96 * (v * n + i):96 * (v * n + i + 1)] for i in range(t)],
                                        wd["ids"][v * n:v * n + t])
                assert u == od_out[v].tobytes(), ("unsafe", v)
                direct["unsafe"] += 1
                if k == 1:
                    rows = eng.pk_cache_add(extra)
                    assert len(set(rows.tolist())) == len(extra) and min(rows.tolist()) >= V * n
                k += 1
        except BaseException as e:  # noqa: BLE001 (reported by the main thread)
            errors.append(e)

    try:
        rows = col.rows(wl["share_pks"])
        th = threading.Thread(target=direct_calls)
        th.start()
        try:
            _, res = collbench_run(col, wl, V, n, t, rows, 4 * V, threads=4)
        finally:
            stop.set()
            th.join(120)
        assert not th.is_alive(), "direct-call thread did not finish"
        assert not errors, errors
        _check(res, V, n, *o)
        assert direct["batch"] >= 3 and direct["unsafe"] >= 3
    finally:
        col.close()


def test_slot_collector_job_over_64_shares(eng):
    """A job of more than 64 shares through SlotCollector.submit (beyond the native collector's
    per-job limit) takes the engine's own batched call for that job alone, on the collector's engine,
    while the collector runs: 3-of-65 with the first two shares invalid == the C oracle (the combine
    of shares 3..5), and a 65-share job beside ordinary ones."""
    V, t, n, R = 2, 3, 65, 1
    wl = bench.make_workload(eng, V, t, n, R, rank=47)
    bad = bench.make_workload(eng, V, t, n, R, rank=48)
    sigs = bytearray(wl["sigs"])
    sigs[0:192] = bad["sigs"][0:192]          # validator 0: shares 1, 2 from another key
    wl["sigs"] = bytes(sigs)
    o_out, o_st, o_err, _ = _oracle(wl, V, t, n)
    small = bench.make_workload(eng, 8, 3, 4, 1, rank=49)
    so_out, so_st, _, _ = _oracle(small, 8, 3, 4)
    with SlotCollector(eng, max_jobs=64, window_s=0.002, in_flight=2) as col:
        futs = []
        for v in range(V):
            futs.append(col.submit(t, ThresholdJob([wl["sigs"][96 * (v * n + i):96 * (v * n + i + 1)] for i in range(n)],
                                                   wl["share_pks"][v * n:(v + 1) * n], wl["ids"][v * n:(v + 1) * n],
                                                   wl["roots"][wl["job_root"][v]])))
        sf = [col.submit(3, ThresholdJob([small["sigs"][96 * (v * 4 + i):96 * (v * 4 + i + 1)] for i in range(4)],
                                         small["share_pks"][v * 4:(v + 1) * 4], small["ids"][v * 4:(v + 1) * 4],
                                         small["roots"][0])) for v in range(8)]
        for v in range(V):
            assert o_st[v] == 0 and futs[v].result(60) == o_out[v].tobytes(), v
        for v in range(8):
            assert so_st[v] == 0 and sf[v].result(60) == so_out[v].tobytes(), v


def test_local_signer_matches_oracle_sign(eng):
    """The local-signing window (ssb_signer_*) behind DvfSigner::local_sign_and_store
    (src/node/dvfcore.rs:241-251; every duty's SecretKey::sign, signing_method.rs:318, selection
    proofs and RANDAO reveals included): 1,536 signatures from 24 concurrent submitters -- 64 shared
    roots (the validators of one attestation committee sign one root) plus 512 roots signed once --
    in several windows; every signature == the C oracle's SecretKey::sign byte for byte, and the
    Ethereum consensus-spec `sign` vector through the window."""
    import hashlib
    from safestakeoperator_amd.collector import LocalSigner
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    shared = [hashlib.sha256(b"duty-root" + i.to_bytes(4, "little")).digest() for i in range(64)]
    work = []
    for i in range(1536):
        sk = 1 + int.from_bytes(hashlib.sha256(b"local-sk" + i.to_bytes(4, "little")).digest(), "big") % (R - 1)
        root = shared[i % 64] if i % 3 else hashlib.sha256(b"own-root" + i.to_bytes(4, "little")).digest()
        work.append((sk, root))
    kat = json.load(open(os.path.join(GOLD, "known_answers.json")))["eth_sign"][0]
    out = {}
    with LocalSigner(eng, max_jobs=512, window_s=0.002) as signer:
        def task(k):
            for i in range(k, len(work), 24):
                out[i] = signer.submit(*work[i])
        th = [threading.Thread(target=task, args=(k,)) for k in range(24)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        kat_sig = signer.sign(int(kat["privkey"], 16), bytes.fromhex(kat["message"]), timeout=60)
        res = {i: f.result(60) for i, f in out.items()}
        signer.flush()
        w, n = signer.stats()
    assert kat_sig.hex() == kat["signature"]
    assert n == len(work) + 1 and w >= 3
    for i, (sk, root) in enumerate(work):
        assert res[i] == bls_c.sign(sk.to_bytes(32, "big"), root), i
