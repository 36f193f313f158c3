"""Per-slot batch collector for threshold aggregation.

The reference aggregates one (validator, duty) at a time: each committee's async `sign` task
collects its operators' partial signatures and calls
`ThresholdSignature::new(t).threshold_aggregate(sigs, pks, ids, msg)` synchronously
(src/validation/impls/hotstuff.rs:141-169; the same call shape in src/crypto/dkg.rs:866-867).
Many such tasks run concurrently, one per validator, and every call pays a full blst verify per
share.

`SlotCollector` is the batched caller that replaces those per-task calls: tasks `submit` their
`ThresholdJob` and get a `concurrent.futures.Future`; one worker thread owns the engine (a context
must not be used from two threads at once, include/ssbls.h) and flushes the pending jobs as ONE
`threshold_aggregate_batch` per distinct threshold when either `max_jobs` are pending or the
oldest pending job has waited `window_s` (the aggregation window), or on `flush()`.  Each future
resolves to exactly what `threshold_aggregate` returns for that job alone: the 96-byte combined
signature, or the reference's `DvfError` raised from `Future.result()`.  Batching changes nothing
observable per job: every job's verify-then-combine is independent, and the RLC batch check falls
back to exact per-share verdicts when any share in the batch is invalid.  The batch's random
linear combination is keyed by a secret the library draws per call (include/ssbls.h), so shares
from different validators' committees cannot be crafted to cancel each other out in one batch.
"""
import threading
import time
from concurrent.futures import Future
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

from .threshold import MAX_T, DvfError, Engine, ThresholdJob, ThresholdSignature, job_shape_error

BatchFn = Callable[[int, Sequence[ThresholdJob]], List[Union[bytes, DvfError]]]


class SlotCollector:
    """Aggregation window over `threshold_aggregate` calls (one worker thread, one engine)."""

    def __init__(self, engine: Optional[Engine] = None, max_jobs: int = 4096, window_s: float = 0.005,
                 batch_fn: Optional[BatchFn] = None):
        if max_jobs < 1 or window_s < 0:
            raise ValueError("max_jobs >= 1 and window_s >= 0")
        self._engine = engine
        self._max = int(max_jobs)
        self._window = float(window_s)
        # batch_fn(t, jobs) -> per-job results; default: the engine's batched entry point
        self._batch_fn = batch_fn or self._engine_batch
        self._cv = threading.Condition()
        self._pending: List[Tuple[int, ThresholdJob, Future, float]] = []
        self._flushing = False                # flush(): drain everything pending without waiting
        self._closed = False
        self.batches: List[int] = []          # sizes of the batches submitted (observability)
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

    def flush(self) -> None:
        """Submit everything pending now and wait until it has been processed."""
        with self._cv:
            futs = [p[2] for p in self._pending]
            if futs:
                self._flushing = True
                self._cv.notify()
        for f in futs:
            f.exception()                     # waits; results stay on the futures

    def close(self) -> None:
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
