"""Per-slot batch collector for threshold aggregation.

The reference aggregates one (validator, duty) at a time: each committee's async `sign` task
collects its operators' partial signatures and calls
`ThresholdSignature::new(t).threshold_aggregate(sigs, pks, ids, msg)` synchronously
(src/validation/impls/hotstuff.rs:141-169; the same call shape in src/crypto/dkg.rs:866-867).
Many such tasks run concurrently, one per validator, and every call pays a full blst verify per
share.

`SlotCollector` is the batched caller that replaces those per-task calls: tasks `submit` their
`ThresholdJob` and get a `concurrent.futures.Future`.  On an engine it runs on the library's native
collector (`NativeCollector`, include/ssbls.h "Per-slot collector", csrc/ssb_collector.hip): the
job's bytes go straight into the open window's pinned buffer, public keys become rows of the
engine's decoded-key table (registered once, `ssb_pk_cache_add`), and up to `in_flight` windows run
on the device while the next fills.  A window closes at `max_jobs` jobs, after `window_s`, or on
`flush()`.  With a `batch_fn` instead (CPU tests), one worker thread runs ONE
`batch_fn(t, jobs)` per distinct threshold of each window.  Each future
resolves to exactly what `threshold_aggregate` returns for that job alone: the 96-byte combined
signature, or the reference's `DvfError` raised from `Future.result()`.  Batching changes nothing
observable per job: every job's verify-then-combine is independent, and the RLC batch check falls
back to exact per-share verdicts when any share in the batch is invalid.  The batch's random
linear combination is keyed by a secret the library draws per call (include/ssbls.h), so shares
from different validators' committees cannot be crafted to cancel each other out in one batch.
"""
import ctypes
import itertools
import threading
import time
from concurrent.futures import Future
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib
from .threshold import (MAX_T, DifferentLength, DvfError, Engine, ThresholdJob, ThresholdSignature, _error_from,
                        job_shape_error)

MAX_JOB_SHARES = 64   # ssb_collector_submit: shares per job


SSB_COLLECTOR_WIRE = 1   # ssb_collector_create2 flag (include/ssbls.h)
WIRE_RECORD = 202        # bincode(bls::Signature)


class NativeCollector:
    """ssb_collector (include/ssbls.h): lock-free submission into pinned windows, one worker thread in
    the library, `in_flight` windows on the device.  It sets the engine's context to one-stream slots
    at depth `in_flight`; the context stays usable by other threads (every library call takes the
    context's lock), so one engine serves the collector and direct calls.  wire=True: the windows
    hold wire records (submit_wire takes the bytes an operator sent; a record that does not
    deserialize makes its share absent, as the reference drops it)."""

    def __init__(self, engine: Engine, max_jobs: int = 4096, max_shares: Optional[int] = None, window_s: float = 0.005,
                 in_flight: int = 20, wire: bool = False):
        self.engine = engine
        self._lib = engine._lib
        self.wire = bool(wire)
        h = ctypes.c_void_p()
        ms = int(max_shares) if max_shares is not None else max(64, 16 * int(max_jobs))
        rc = self._lib.ssb_collector_create2(engine.handle, int(max_jobs), ms, int(round(window_s * 1e6)),
                                             int(in_flight), SSB_COLLECTOR_WIRE if wire else 0, ctypes.byref(h))
        if rc != 0:
            raise RuntimeError("ssb_collector_create failed (%d): %s" % (rc, self._lib.ssb_last_error(engine.handle)))
        self._h = h
        self._rows: Dict[bytes, int] = {}
        self._rows_lock = threading.Lock()

    @property
    def handle(self):
        return self._h

    def rows(self, pks: Sequence[bytes]) -> np.ndarray:
        """Key-table rows of these public keys, registering the ones not seen before."""
        with self._rows_lock:
            new = [p for p in dict.fromkeys(bytes(p) for p in pks) if p not in self._rows]
            if new:
                buf = np.frombuffer(b"".join(new), dtype=np.uint8)
                idx = np.zeros(len(new), dtype=np.uint32)
                rc = self._lib.ssb_collector_register_keys(self._h, len(new), buf.ctypes.data_as(_lib._u8p),
                                                           idx.ctypes.data_as(_lib._u32p))
                if rc != 0:
                    raise RuntimeError("ssb_collector_register_keys failed (%d)" % rc)
                self._rows.update(zip(new, idx.tolist()))
            return np.fromiter((self._rows[bytes(p)] for p in pks), dtype=np.uint32, count=len(pks))

    def submit(self, t: int, sig96: np.ndarray, rows: np.ndarray, ids: np.ndarray, root: bytes, result: "_lib.JobResult",
               cb=None, user: int = 0) -> None:
        """One job (arrays already packed: sig96 uint8[n*96], rows uint32[n], ids uint64[n]); `result`
        and the arrays stay alive until the job is done."""
        n = len(ids)
        rc = self._lib.ssb_collector_submit(self._h, int(t), n, sig96.ctypes.data if n else None,
                                            rows.ctypes.data if n else None, ids.ctypes.data if n else None,
                                            root, ctypes.addressof(result), cb, ctypes.c_void_p(user))
        if rc != 0:
            raise RuntimeError("ssb_collector_submit failed (%d)" % rc)

    def submit_wire(self, t: int, records: Sequence[bytes], rows: np.ndarray, ids: np.ndarray, root: bytes,
                    result: "_lib.JobResult", cb=None, user: int = 0) -> None:
        """One job whose shares are wire records as received (a wire collector); the records are copied
        before this returns."""
        n = len(ids)
        bufs = [bytes(r) for r in records]
        ptrs = (ctypes.c_char_p * max(1, n))(*bufs) if n else (ctypes.c_char_p * 1)()
        lens = (ctypes.c_size_t * max(1, n))(*[len(b) for b in bufs])
        rc = self._lib.ssb_collector_submit_wire(self._h, int(t), n, ctypes.cast(ptrs, ctypes.c_void_p),
                                                 ctypes.cast(lens, ctypes.c_void_p), rows.ctypes.data if n else None,
                                                 ids.ctypes.data if n else None, root, ctypes.addressof(result), cb,
                                                 ctypes.c_void_p(user))
        if rc != 0:
            raise RuntimeError("ssb_collector_submit_wire failed (%d)" % rc)

    def wait(self, result: "_lib.JobResult") -> None:
        self._lib.ssb_collector_wait(self._h, ctypes.addressof(result))

    def flush(self) -> None:
        self._lib.ssb_collector_flush(self._h)

    def stats(self) -> Tuple[int, int, int]:
        w, j, s = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._lib.ssb_collector_stats(self._h, ctypes.byref(w), ctypes.byref(j), ctypes.byref(s))
        return int(w.value), int(j.value), int(s.value)

    def profile(self) -> dict:
        """Worker-thread profile: ms closing + launching windows, delivering, waiting on the device;
        submits that waited for a new window."""
        a, b, c, w = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        self._lib.ssb_collector_profile(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(w))
        return dict(seal_ms=round(a.value, 3), deliver_ms=round(b.value, 3), backpressure_ms=round(c.value, 3),
                    full_waits=int(w.value))

    def close(self) -> None:
        if self._h:
            self._lib.ssb_collector_destroy(self._h)   # drains every submitted job
            self._h = None


def result_of(r: "_lib.JobResult") -> Union[bytes, DvfError, Exception]:
    """The job's threshold_aggregate outcome from its ssb_job_result."""
    if r.status == 0:
        return bytes(r.sig96)
    return _error_from(int(r.status), int(r.err[0]), int(r.err[1]))

class LocalSigner:
    """The local-signing window (include/ssbls.h, ssb_signer_*): the batched form of
    `DvfSigner::local_sign_and_store`'s `SecretKey::sign` (src/node/dvfcore.rs:241-251), which every
    duty of every validator reaches once (src/validation/signing_method.rs:318 -- attestations, blocks,
    aggregates, selection proofs and RANDAO reveals).  `submit(sk, root)` returns a Future of the
    96-byte signature; the library's worker signs each window with one ssb_sign_batch (every distinct
    root hashed once).  Mirrors rust/src/validation/impls/slot_signer.rs."""

    def __init__(self, engine: Engine, max_jobs: int = 4096, window_s: float = 0.002):
        self.engine = engine
        self._lib = engine._lib
        h = ctypes.c_void_p()
        rc = self._lib.ssb_signer_create(engine.handle, int(max_jobs), int(round(window_s * 1e6)), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError("ssb_signer_create failed (%d)" % rc)
        self._h = h
        self._ids = itertools.count(1)
        self._inflight: Dict[int, Tuple[Future, "_lib.SignResult"]] = {}
        self._cb = _lib.SIGN_DONE_FN(self._done)   # kept alive as long as the signer

    def submit(self, sk: int, root: bytes) -> Future:
        if not 0 < int(sk) < (1 << 255) or len(root) != 32:
            raise ValueError("a secret scalar in (0, r) and a 32-byte signing root")
        fut: Future = Future()
        res = _lib.SignResult()
        key = next(self._ids)
        self._inflight[key] = (fut, res)
        skb = int(sk).to_bytes(32, "little")
        rc = self._lib.ssb_signer_submit(self._h, skb, bytes(root), ctypes.addressof(res), self._cb, ctypes.c_void_p(key))
        if rc != 0:
            self._inflight.pop(key, None)
            raise RuntimeError("ssb_signer_submit failed (%d)" % rc)
        return fut

    def sign(self, sk: int, root: bytes, timeout: Optional[float] = None) -> bytes:
        """SecretKey::sign(root), blocking."""
        return self.submit(sk, root).result(timeout)

    def _done(self, user, res_p) -> None:
        """ssb_sign_done_fn, on the library's worker thread."""
        fut, res = self._inflight.pop(int(user or 0))
        if not fut.set_running_or_notify_cancel():
            return
        if res.rc == 0:
            fut.set_result(bytes(res.sig96))
        else:
            fut.set_exception(RuntimeError("ssb_sign_batch failed (%d)" % res.rc))

    def flush(self) -> None:
        self._lib.ssb_signer_flush(self._h)

    def stats(self) -> Tuple[int, int]:
        w, n = ctypes.c_uint64(), ctypes.c_uint64()
        self._lib.ssb_signer_stats(self._h, ctypes.byref(w), ctypes.byref(n))
        return int(w.value), int(n.value)

    def close(self) -> None:
        if self._h:
            self._lib.ssb_signer_destroy(self._h)   # signs and delivers every submission
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


BatchFn = Callable[[int, Sequence[ThresholdJob]], List[Union[bytes, DvfError]]]


class SlotCollector:
    """Aggregation window over `threshold_aggregate` calls: the engine's native collector, or (with a
    `batch_fn`, CPU tests) one Python worker thread calling batch_fn per window and threshold."""

    def __init__(self, engine: Optional[Engine] = None, max_jobs: int = 4096, window_s: float = 0.005,
                 batch_fn: Optional[BatchFn] = None, in_flight: int = 20):
        if max_jobs < 1 or window_s < 0:
            raise ValueError("max_jobs >= 1 and window_s >= 0")
        self._engine = engine
        self._max = int(max_jobs)
        self._window = float(window_s)
        self._native: Optional[NativeCollector] = None
        self.batches: List[int] = []          # sizes of the batches submitted (observability)
        if batch_fn is None:
            from .threshold import default_engine
            self._native = NativeCollector(engine or default_engine(), max_jobs=max_jobs, window_s=window_s,
                                           in_flight=in_flight)
            self._inflight: Dict[int, Tuple[Future, "_lib.JobResult", tuple]] = {}
            self._ids = itertools.count(1)
            self._cb = _lib.JOB_DONE_FN(self._done)   # kept alive as long as the collector
            self._closed = False
            return
        self._batch_fn = batch_fn
        self._cv = threading.Condition()
        self._pending: List[Tuple[int, ThresholdJob, Future, float]] = []
        self._flushing = False                # flush(): drain everything pending without waiting
        self._closed = False
        self._worker = threading.Thread(target=self._run, name="ssb-slot-collector", daemon=True)
        self._worker.start()

    # -- the replacement for ThresholdSignature::new(t).threshold_aggregate(...) per task --
    def submit(self, threshold: int, job: ThresholdJob) -> Future:
        """A future of this job's result.  A job the engine cannot take (threshold outside
        [1, MAX_T], a malformed message / signature / key) fails alone, at once, and never joins
        a batch: the other validators of the slot are unaffected."""
        fut: Future = Future()
        bad = None
        if not 1 <= int(threshold) <= MAX_T:
            bad = "threshold must be in [1, %d]" % MAX_T
        elif len(job.sigs) == len(job.pks) == len(job.ids):   # DifferentLength: the engine's own error
            bad = job_shape_error(job)
        if bad:
            fut.set_running_or_notify_cancel()
            fut.set_exception(ValueError(bad))
            return fut
        if self._native is not None:
            return self._submit_native(int(threshold), job, fut)
        with self._cv:
            if self._closed:
                raise RuntimeError("collector closed")
            self._pending.append((int(threshold), job, fut, time.monotonic()))
            if len(self._pending) >= self._max:
                self._cv.notify()
            elif len(self._pending) == 1:
                self._cv.notify()             # start the window
        return fut

    def threshold_aggregate(self, threshold: int, sigs: Sequence[bytes], pks: Sequence[bytes], ids: Sequence[int],
                            msg: bytes, timeout: Optional[float] = None) -> bytes:
        """Blocking form with the reference's signature and error behaviour."""
        return self.submit(threshold, ThresholdJob(sigs, pks, ids, msg)).result(timeout)

    # -- native path --
    def _submit_native(self, t: int, job: ThresholdJob, fut: Future) -> Future:
        # the reference's two length checks (generic_threshold.rs:133-138), before the engine
        if len(job.sigs) != len(job.pks):
            return self._fail(fut, DifferentLength(len(job.sigs), len(job.pks)))
        if len(job.sigs) != len(job.ids):
            return self._fail(fut, DifferentLength(len(job.sigs), len(job.ids)))
        if len(job.sigs) > MAX_JOB_SHARES:
            # beyond the collector's per-job limit: the engine's own batched call for this job alone, as
            # slot_collector.rs falls back to the per-job call (the reference returns a result here too)
            fut.set_running_or_notify_cancel()
            try:
                r = ThresholdSignature(t, self._native.engine).threshold_aggregate_batch([job])[0]
            except BaseException as e:
                fut.set_exception(e)
                return fut
            if isinstance(r, (DvfError, ValueError)):
                fut.set_exception(r)
            else:
                fut.set_result(r)
            return fut
        if self._closed:
            raise RuntimeError("collector closed")
        n = len(job.sigs)
        sig = np.frombuffer(b"".join(bytes(s) for s in job.sigs), dtype=np.uint8) if n else np.zeros(1, np.uint8)
        rows = self._native.rows(job.pks) if n else np.zeros(1, np.uint32)
        ids = np.asarray([int(i) for i in job.ids], dtype=np.uint64) if n else np.zeros(1, np.uint64)
        if not n:
            ids = ids[:0]
        root = bytes(job.msg)
        res = _lib.JobResult()
        key = next(self._ids)
        self._inflight[key] = (fut, res, (sig, rows, ids, root))   # alive until delivered
        try:
            self._native.submit(t, sig, rows, ids, root, res, self._cb, key)
        except BaseException:
            self._inflight.pop(key, None)
            raise
        return fut

    @staticmethod
    def _fail(fut: Future, e: Exception) -> Future:
        fut.set_running_or_notify_cancel()
        fut.set_exception(e)
        return fut

    def _done(self, user, res_p) -> None:
        """ssb_job_done_fn, on the library's worker thread."""
        fut, res, _ = self._inflight.pop(int(user or 0))
        if not fut.set_running_or_notify_cancel():
            return
        r = result_of(res)
        if isinstance(r, Exception):
            fut.set_exception(r)
        else:
            fut.set_result(r)

    def flush(self) -> None:
        """Submit everything pending now and wait until it has been processed."""
        if self._native is not None:
            self._native.flush()
            return
        with self._cv:
            futs = [p[2] for p in self._pending]
            if futs:
                self._flushing = True
                self._cv.notify()
        for f in futs:
            f.exception()                     # waits; results stay on the futures

    def close(self) -> None:
        if self._native is not None:
            if not self._closed:
                self._closed = True
                self._native.flush()
                self.native_stats = self._native.stats()   # (windows, jobs, shares)
                self._native.close()
            return
        with self._cv:
            self._closed = True
            self._cv.notify()
        self._worker.join()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- worker --
    def _engine_batch(self, t: int, jobs: Sequence[ThresholdJob]) -> List[Union[bytes, DvfError]]:
        return ThresholdSignature(t, self._engine).threshold_aggregate_batch(jobs)

    def _take(self) -> List[Tuple[int, ThresholdJob, Future, float]]:
        """Wait for a full batch, an expired window, a flush or close; return the jobs to run."""
        with self._cv:
            while True:
                if self._pending:
                    full = len(self._pending) >= self._max
                    waited = time.monotonic() - self._pending[0][3]
                    if full or waited >= self._window or self._flushing or self._closed:
                        batch, self._pending = self._pending[:self._max], self._pending[self._max:]
                        if not self._pending:
                            self._flushing = False
                        return batch
                    self._cv.wait(self._window - waited)
                elif self._closed:
                    return []
                else:
                    self._cv.wait()

    def _run(self) -> None:
        while True:
            batch = self._take()
            if not batch:
                return
            self.batches.append(len(batch))
            by_t: Dict[int, List[Tuple[ThresholdJob, Future]]] = {}
            for t, job, fut, _ in batch:
                by_t.setdefault(t, []).append((job, fut))
            for t, items in by_t.items():
                live = [(j, f) for j, f in items if f.set_running_or_notify_cancel()]
                if not live:
                    continue
                try:
                    res = self._batch_fn(t, [j for j, _ in live])
                except BaseException as e:    # engine failure: every job of the batch sees it
                    for _, f in live:
                        f.set_exception(e)
                    continue
                for (_, f), r in zip(live, res):
                    if isinstance(r, (DvfError, ValueError)):
                        f.set_exception(r)
                    else:
                        f.set_result(r)


# numpy view of ssb_job_result (include/ssbls.h), for arrays of results filled by native code
JOB_RESULT_DTYPE = np.dtype([("sig96", np.uint8, 96), ("err", "<u8", 2), ("verdicts", "<u8"), ("status", "<i4"),
                             ("rc", "<i4"), ("n_shares", "<u4"), ("done", "<u4"), ("absent", "<u8")], align=True)
assert JOB_RESULT_DTYPE.itemsize == ctypes.sizeof(_lib.JobResult)


def wire_records(sigs: bytes) -> bytes:
    """bincode(bls::Signature) of each 96-byte compressed signature: u64 LE length 194, "0x", 192
    lowercase hex digits -- the bytes an operator sends (src/node/dvfcore.rs:245-251)."""
    n = len(sigs) // 96
    a = np.frombuffer(sigs, dtype=np.uint8).reshape(n, 96)
    hx = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
    out = np.empty((n, WIRE_RECORD), dtype=np.uint8)
    out[:, :8] = np.frombuffer((194).to_bytes(8, "little"), dtype=np.uint8)
    out[:, 8], out[:, 9] = ord("0"), ord("x")
    out[:, 10::2] = hx[a >> 4]
    out[:, 11::2] = hx[a & 15]
    return out.tobytes()


def collbench_run(col: NativeCollector, wl: dict, V: int, n: int, t: int, rows: np.ndarray, n_jobs: int,
                  threads: int = 8, wire: Optional[bytes] = None) -> Tuple[float, np.ndarray]:
    """bench_tools/libcollbench.so: `threads` native submitters push n_jobs jobs (job k = validator
    k % V of the workload) through the collector; (seconds first submit -> last result, results).
    wire: the workload's shares as wire records (wire_records), submitted with
    ssb_collector_submit_wire to a wire collector."""
    import os
    from .build import build_collbench
    lib = ctypes.CDLL(build_collbench(verbose=False))
    fn = lib.ssb_collbench_run_wire if wire is not None else lib.ssb_collbench_run
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.POINTER(ctypes.c_double)]
    sig = np.frombuffer(wire if wire is not None else wl["sigs"], dtype=np.uint8)
    ids = np.asarray(wl["ids"], dtype=np.uint64)
    roots = np.frombuffer(b"".join(wl["roots"]), dtype=np.uint8)
    jr = np.asarray(wl["job_root"], dtype=np.uint32)
    rows = np.ascontiguousarray(rows, dtype=np.uint32)
    res = np.zeros(n_jobs, dtype=JOB_RESULT_DTYPE)
    sec = ctypes.c_double()
    rc = fn(col.handle, int(threads), int(n_jobs), V, n, t, sig.ctypes.data, rows.ctypes.data, ids.ctypes.data,
            roots.ctypes.data, jr.ctypes.data, res.ctypes.data, ctypes.byref(sec))
    if rc != 0:
        raise RuntimeError("ssb_collbench_run failed (%d)" % rc)
    return float(sec.value), res
