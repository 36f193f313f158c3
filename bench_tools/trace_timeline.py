"""Timeline analysis of a `rocprofv3 --kernel-trace --output-format csv` run of bench.py.

    python bench_tools/trace_timeline.py gpurun_out/<tag>/raw/kt_kernel_trace.csv [--first-batch 5 --batches 20]

Batches are delimited by the decode kernel (one k_decode_sig / k_decode2 per batch).  For the
window from batch `first` start to the end of the last kernel of batch first+batches-1 it prints:
per-kernel dispatch count / busy time / mean duration, per-queue busy fraction, the time-average
number of kernels running and of waves resident (grid / 64, capped by the kernel's occupancy
bound from its VGPR count), and the batch latencies (decode start -> combine end).
"""
import argparse
import collections
import csv


def occupancy(vgpr, agpr):
    regs = max(vgpr + agpr, 1)
    return max(1, min(8, 512 // regs))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--first-batch", type=int, default=5)
    ap.add_argument("--batches", type=int, default=20)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        name = r["Kernel_Name"].split("(")[0].replace("ssb::k::", "")
        rows.append(dict(name=name, q=int(r["Queue_Id"]), t0=int(r["Start_Timestamp"]), t1=int(r["End_Timestamp"]),
                         waves=(int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) + 63) // 64,
                         occ=occupancy(int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"])),
                         lds=int(r["LDS_Block_Size"]), scratch=int(r["Scratch_Size"])))
    rows.sort(key=lambda r: r["t0"])
    dec = [r for r in rows if r["name"] in ("k_decode_sig", "k_decode2", "k_decode")]
    fb, lb = a.first_batch, a.first_batch + a.batches - 1
    if len(dec) <= lb:
        raise SystemExit("only %d decode dispatches" % len(dec))
    w0 = dec[fb]["t0"]
    # end: the last combine-side kernel that starts before the next (untimed) batch's decode
    nxt = dec[lb + 1]["t0"] if len(dec) > lb + 1 else float("inf")
    in_win = [r for r in rows if w0 <= r["t0"] < nxt]
    w1 = max(r["t1"] for r in in_win)
    span = (w1 - w0) / 1e6
    print("window: batches %d..%d, %.3f ms (%.3f ms/batch)" % (fb, lb, span, span / a.batches))
    agg = collections.defaultdict(lambda: [0, 0.0, 0, 0])
    for r in in_win:
        g = agg[r["name"]]
        g[0] += 1
        g[1] += (r["t1"] - r["t0"]) / 1e6
        g[2] = r["waves"]
        g[3] = r["occ"]
    print("%-34s %5s %9s %8s %6s %4s" % ("kernel", "n", "busy_ms", "mean_ms", "waves", "occ"))
    for k, (n, busy, wv, oc) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-34s %5d %9.2f %8.3f %6d %4d" % (k, n, busy, busy / n, wv, oc))
    qb = collections.defaultdict(float)
    for r in in_win:
        qb[r["q"]] += (min(r["t1"], w1) - max(r["t0"], w0)) / 1e6
    print("queues: %d; busy fraction per queue: %s" % (len(qb), " ".join("%.2f" % (v / span) for v in sorted(qb.values(), reverse=True))))
    # time-average running kernels and resident waves (waves capped by 1024 SIMDs x occupancy)
    ev = []
    for r in in_win:
        slots = r["waves"] / r["occ"]                  # SIMD-slots the kernel would fill
        ev.append((r["t0"], 1, slots))
        ev.append((r["t1"], -1, -slots))
    ev.sort()
    t_prev, k_run, s_run, k_int, s_int, sat = w0, 0, 0.0, 0.0, 0.0, 0.0
    for t, dk, ds in ev:
        t = min(max(t, w0), w1)
        dt = (t - t_prev) / 1e6
        k_int += k_run * dt
        s_int += min(s_run, 1024.0) * dt
        if s_run >= 1024:
            sat += dt
        k_run += dk
        s_run += ds
        t_prev = t
    print("mean kernels running %.1f; mean SIMD-slot demand %.0f of 1024 (capped); saturated %.0f%% of the window"
          % (k_int / span, s_int / span, 100 * sat / span))
    # per-batch latency: decode start -> last kernel before the next decode on the same queue chain
    lat = []
    for b in range(fb, lb + 1):
        q = dec[b]["q"]
        t_end = dec[b]["t1"]
        for r in rows:
            if r["q"] == q and r["t0"] >= dec[b]["t0"] and (b + 1 >= len(dec) or r["t0"] < max(
                    (d["t0"] for d in dec[b + 1:] if d["q"] == q), default=float("inf"))):
                t_end = max(t_end, r["t1"])
        lat.append((t_end - dec[b]["t0"]) / 1e6)
    print("batch latency on its slot queue (ms): " + " ".join("%.1f" % x for x in lat))


if __name__ == "__main__":
    main()
