"""Critical path inside k_fb_excl for ONE failed C2 batch (one-stream slot, depth 1): the experiment
build with trace stamps (round 5),
    SSB_VARIANT=trace SSB_VARIANT_DEFS=-DSSB_TRACE_TAIL python -m safestakeoperator_amd.build
    SSB_LIB_VARIANT=trace python bench_tools/trace_fb.py {one|pct|badop} > gpurun_out/<tag>/fb_<pattern>.txt
Prints, per traced stage of the third batch, the record count and the first start / last end (us
from the first traced block), and the distribution of per-record (end - block start)."""
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
TAGS = {10: "ex_item", 11: "ex_group_comb", 12: "ex_group_check", 13: "ex_single", 14: "ex_pair_x", 15: "ex_final",
        16: "ex_pair_root", 17: "ex_quarter_sum"}


def main(pattern):
    import numpy as np
    import torch
    import bench
    from safestakeoperator_amd import Engine, DST, _lib
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    V, t, n, R = 4096, 3, 4, 64
    kw = dict(one=dict(invalid_count=1), pct=dict(invalid_rate=0.01), badop=dict(bad_operator=1))[pattern]
    wl = bench.make_workload(eng, V, t, n, R, 0, **kw)
    N = V * n
    lib = eng._lib
    pk = np.frombuffer(wl["pks"], dtype=np.uint8)
    assert lib.ssb_pk_cache_set(eng.handle, N, pk.ctypes.data_as(_lib._u8p)) == 0
    assert lib.ssb_set_slot_streams(eng.handle, 1) == 0 and lib.ssb_set_pipeline_depth(eng.handle, 1) == 0
    u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_sig, d_roots = u8(wl["sigs"]), u8(b"".join(wl["roots"]))
    d_idx = torch.arange(0, N, dtype=torch.int32, device=dev)
    d_ids = torch.tensor(wl["ids"], dtype=torch.int64, device=dev)
    d_off = torch.arange(0, N + 1, n, dtype=torch.int32, device=dev)
    d_t = torch.full((V,), t, dtype=torch.int32, device=dev)
    d_jr = torch.tensor(wl["job_root"], dtype=torch.int32, device=dev)
    out = torch.empty((V, 96), dtype=torch.uint8, device=dev)
    st = torch.empty((V,), dtype=torch.int32, device=dev)
    err = torch.empty((V, 2), dtype=torch.int64, device=dev)
    ver = torch.empty((N,), dtype=torch.uint8, device=dev)
    dst = (ctypes.c_uint8 * len(DST)).from_buffer_copy(DST)
    s = ctypes.c_void_p(lib.ssb_slot_stream(eng.handle, 0))
    buf = (ctypes.c_ulonglong * (4 * 2048))()
    traced = hasattr(lib, "ssb_debug_trace_bisect")   # (the product library: verdicts only)
    if traced:
        lib.ssb_debug_trace_bisect(buf)   # clear
    valid = np.asarray(wl["valid"], dtype=np.uint8)
    for i in range(3):
        rc = lib.ssb_threshold_aggregate_batch_cached_dev(eng.handle, V, N, d_off.data_ptr(), d_t.data_ptr(), d_sig.data_ptr(),
                                                          d_idx.data_ptr(), d_ids.data_ptr(), d_jr.data_ptr(), R, d_roots.data_ptr(),
                                                          ctypes.cast(dst, _lib._u8p), len(DST), 5 + i, out.data_ptr(),
                                                          st.data_ptr(), err.data_ptr(), ver.data_ptr(), s)
        assert rc == 0, lib.ssb_last_error(eng.handle)
        torch.cuda.synchronize()
        ok = bool((ver.cpu().numpy() == valid).all())
        if not traced:
            print("batch %d verdicts_ok %s" % (i, ok))
            continue
        m = lib.ssb_debug_trace_bisect(buf)
        if i < 2:
            continue
        rows = [(TAGS.get(buf[4 * k], "?"), buf[4 * k + 1], buf[4 * k + 2], buf[4 * k + 3]) for k in range(max(m, 0))]
        print("pattern %s verdicts_ok %s records %d" % (pattern, ok, len(rows)))
        if not rows:
            return
        t0 = min(r[2] for r in rows)
        agg = collections.defaultdict(list)
        for tag, blk, a, e in rows:
            agg[tag].append((blk, (a - t0) / 100.0, (e - t0) / 100.0))
        for tag, v in sorted(agg.items(), key=lambda x: max(y[2] for y in x[1])):
            ends = sorted(y[2] for y in v)
            per = sorted(y[2] - y[1] for y in v)
            print("  %-15s n %4d  first end %9.1f us  median end %9.1f  last end %9.1f  (end - block start: median %9.1f max %9.1f)"
                  % (tag, len(v), ends[0], ends[len(ends) // 2], ends[-1], per[len(per) // 2], per[-1]))
    eng.close()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "badop")
