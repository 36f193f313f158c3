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
