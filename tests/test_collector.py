"""SlotCollector: the per-slot aggregation window over threshold_aggregate.

CPU tests drive the collector with a batch function built on the oracle (the reference scan +
combine per job), so windowing, routing of results and errors, per-threshold grouping and
concurrency are checked without a GPU; the GPU test runs it on the engine against the golden
threshold cases."""
import json
import os
import threading

import pytest

from safestakeoperator_amd import DvfError, SlotCollector, ThresholdJob
from safestakeoperator_amd.threshold import _error_from

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cases():
    with open(os.path.join(GOLD, "threshold_cases.json")) as f:
        return json.load(f)["cases"]


def _job(c):
    return ThresholdJob([bytes.fromhex(s) for s in c["sigs"]], [bytes.fromhex(p) for p in c["pks"]], c["ids"],
                        bytes.fromhex(c["root"]))


def _expected(c):
    if c["expected_status"] == 0:
        return bytes.fromhex(c["master_sig"])
    pl = c["expected_payload"]
    return _error_from(c["expected_status"], pl[0], pl[1] if len(pl) > 1 else 0)


def _golden_batch_fn(calls):
    """batch function answering from the golden expectations (keyed by the job's content)"""
    table = {}
    for c in _cases():
        j = _job(c)
        table[(c["t"], tuple(j.sigs), tuple(j.pks), tuple(j.ids), j.msg)] = _expected(c)

    def fn(t, jobs):
        calls.append((t, len(jobs)))
        return [table[(t, tuple(j.sigs), tuple(j.pks), tuple(j.ids), j.msg)] for j in jobs]
    return fn


def _check(fut, want):
    if isinstance(want, DvfError):
        with pytest.raises(DvfError) as ei:
            fut.result(10)
        assert ei.value == want
    else:
        assert fut.result(10) == want


def test_window_batches_and_routes_results():
    calls = []
    cases = _cases()
    with SlotCollector(max_jobs=1000, window_s=0.05, batch_fn=_golden_batch_fn(calls)) as col:
        futs = [(col.submit(c["t"], _job(c)), _expected(c)) for c in cases]
        for f, want in futs:
            _check(f, want)
    # one window: one batch call per distinct threshold
    assert sum(n for _, n in calls) == len(cases)
    assert len(calls) == len({c["t"] for c in cases})


def test_max_jobs_splits_batches():
    calls = []
    cases = [c for c in _cases() if c["t"] == 3]
    with SlotCollector(max_jobs=2, window_s=10.0, batch_fn=_golden_batch_fn(calls)) as col:
        futs = [(col.submit(3, _job(c)), _expected(c)) for c in cases]
        col.flush()
        for f, want in futs:
            _check(f, want)
    assert all(n <= 2 for _, n in calls) and sum(n for _, n in calls) == len(cases)


def test_flush_does_not_wait_for_window():
    calls = []
    c = [c for c in _cases() if c["expected_status"] == 0][0]
    col = SlotCollector(max_jobs=100, window_s=30.0, batch_fn=_golden_batch_fn(calls))
    try:
        f = col.submit(c["t"], _job(c))
        col.flush()
        assert f.done() and f.result() == _expected(c)
    finally:
        col.close()


def test_concurrent_submitters():
    calls = []
    cases = _cases()
    out = {}
    with SlotCollector(max_jobs=64, window_s=0.02, batch_fn=_golden_batch_fn(calls)) as col:
        def task(k):
            c = cases[k % len(cases)]
            try:
                out[k] = col.threshold_aggregate(c["t"], *(lambda j: (j.sigs, j.pks, j.ids, j.msg))(_job(c)))
            except DvfError as e:
                out[k] = e
        th = [threading.Thread(target=task, args=(k,)) for k in range(200)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    for k, r in out.items():
        assert r == _expected(cases[k % len(cases)])
    assert len(out) == 200


def test_engine_failure_reaches_every_job():
    def boom(t, jobs):
        raise RuntimeError("device lost")
    with SlotCollector(max_jobs=8, window_s=0.01, batch_fn=boom) as col:
        f = col.submit(3, _job(_cases()[0]))
        with pytest.raises(RuntimeError):
            f.result(10)


@pytest.mark.gpu
def test_collector_on_engine():
    """SlotCollector on its own engine (the native collector takes a context over)."""
    from safestakeoperator_amd import Engine
    cases = _cases()
    with Engine(0) as eng:
        with SlotCollector(eng, max_jobs=4096, window_s=0.01, in_flight=2) as col:
            futs = [(col.submit(c["t"], _job(c)), _expected(c)) for c in cases for _ in range(3)]
            for f, want in futs:
                _check(f, want)


def test_malformed_job_fails_alone():
    """A job with a short message, a wrong-length signature or an out-of-range threshold fails
    its own future at submit and never joins the batch; the slot's other jobs aggregate."""
    calls = []
    cases = [c for c in _cases() if c["expected_status"] == 0][:3]
    with SlotCollector(max_jobs=64, window_s=0.01, batch_fn=_golden_batch_fn(calls)) as col:
        good = [col.submit(c["t"], _job(c)) for c in cases]
        j = _job(cases[0])
        bad_msg = col.submit(cases[0]["t"], ThresholdJob(j.sigs, j.pks, j.ids, b"\0" * 31))
        bad_sig = col.submit(cases[0]["t"], ThresholdJob([s[:95] for s in j.sigs], j.pks, j.ids, j.msg))
        bad_t = col.submit(0, j)
        for f in (bad_msg, bad_sig, bad_t):
            with pytest.raises(ValueError):
                f.result(1)
        for c, f in zip(cases, good):
            _check(f, _expected(c))
    assert sum(n for _, n in calls) == len(cases)
