"""Diagnostic (round 5): registry-id batches through the cached one-stream path, timed, at growing
sizes and invalid counts, verdicts/statuses against the construction truth (no oracle).
    python bench_tools/r05_diag.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from safestakeoperator_amd import Engine  # noqa: E402
from test_gpu_configs import _cached_one_stream  # noqa: E402

t, n = 3, 4
cases = [(64, 4, 0, "registry"), (64, 4, 1, "registry"), (4096, 64, 0, "registry"), (4096, 64, 1, "seq"),
         (4096, 64, 1, "registry")]
if len(sys.argv) > 1:   # V R invalid ids
    cases = [(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])]
with Engine(0) as eng:
    for V, R, inv, ids in cases:
        wl = bench.make_workload(eng, V, t, n, R, rank=21, ids=ids, invalid_count=inv)
        print("V %d inv %d %s: workload ready" % (V, inv, ids), flush=True)
        t0 = time.time()
        runs = _cached_one_stream(eng, wl, V, t, n, slots=1)
        dt = time.time() - t0
        out, st, err, ver = runs[0]
        valid = np.asarray(wl["valid"], dtype=np.uint8)
        print("V %d inv %d %s: %.3f s, verdicts ok %s, statuses %s" % (V, inv, ids, dt, bool((ver == valid).all()),
                                                                     np.unique(st, return_counts=True)), flush=True)
