"""Critical path inside the fused tail launches of ONE C2 batch (one-stream slot, depth 1): needs the
experiment build with trace stamps,
    SSB_VARIANT=trace SSB_VARIANT_DEFS=-DSSB_TRACE_TAIL python -m safestakeoperator_amd.build
    SSB_LIB_VARIANT=trace python bench_tools/trace_tail.py > gpurun_out/<tag>/trace.txt
Prints, per traced stage, the block count and the first start / last end (us from the first
traced block) of each of three batches, plus the hipEvent times of every stage."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def main():
    import numpy as np
    import torch
    import bench
    from safestakeoperator_amd import Engine, DST, _lib
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(eng, V, t, n, R, 0)
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
    TAGS = {1: "w2_g2window", 2: "w2_g1window", 3: "w2_g1horner", 4: "w2_h2cclear", 5: "w2_h2caffine",
            6: "mf_miller", 7: "mf_group", 8: "mf_product", 9: "mf_final"}
    buf = (ctypes.c_ulonglong * (4 * 2048))()
    for fn in ("ssb_debug_trace_msm", "ssb_debug_trace_pair"):
        getattr(lib, fn)(buf)   # clear
    for i in range(3):
        if i == 2:
            eng.kernel_timing(True)
        rc = lib.ssb_threshold_aggregate_batch_cached_dev(eng.handle, V, N, d_off.data_ptr(), d_t.data_ptr(), d_sig.data_ptr(),
                                                          d_idx.data_ptr(), d_ids.data_ptr(), d_jr.data_ptr(), R, d_roots.data_ptr(),
                                                          ctypes.cast(dst, _lib._u8p), len(DST), 5 + i, out.data_ptr(),
                                                          st.data_ptr(), err.data_ptr(), ver.data_ptr(), s)
        assert rc == 0, lib.ssb_last_error(eng.handle)
        torch.cuda.synchronize()
        os.write(1, b"BATCH %d ok=%d\n" % (i, int(bool((st == 0).all().item()) and bool(ver.all().item()))))
        for fn in ("ssb_debug_trace_msm", "ssb_debug_trace_pair"):
            m = getattr(lib, fn)(buf)
            for k in range(max(m, 0)):
                os.write(1, b"TRACE %s %d %d %d\n" % (TAGS.get(buf[4 * k], "?").encode(), buf[4 * k + 1], buf[4 * k + 2],
                                                      buf[4 * k + 3]))
    for k in ("k_decode", "k_subgroup", "k_msm_g2", "k_miller", "k_fallback_verify", "k_combine_fast"):
        tot, cnt = eng.kernel_time(k)
        os.write(1, b"EVENT %s %.4f ms\n" % (k.encode(), tot / max(cnt, 1)))
    eng.close()


def summarize(path):
    import collections
    lines = open(path).read().split("\n")
    cur, batches = None, collections.defaultdict(list)
    for ln in lines:
        if ln.startswith("BATCH"):
            cur = ln
        elif ln.startswith("TRACE") and cur:
            f = ln.split()
            batches[cur].append((f[1], int(f[2]), int(f[3]), int(f[4])))
    for b, rows in batches.items():
        if not rows:
            continue
        t0 = min(r[2] for r in rows)
        agg = collections.defaultdict(lambda: [0, 1 << 62, 0])
        for tag, _, a, e in rows:
            g = agg[tag]
            g[0] += 1; g[1] = min(g[1], a); g[2] = max(g[2], e)
        print(b)
        for tag, (c, a, e) in sorted(agg.items(), key=lambda x: x[1][2]):
            print("  %-14s blocks %4d  first start %8.1f us  last end %8.1f us" % (tag, c, (a - t0) / 100.0, (e - t0) / 100.0))
    for ln in lines:
        if ln.startswith("EVENT"):
            print(ln)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        main()
