"""Device timeline of the timed run of `SSB_DEBUG_GATE=1 rocprofv3 --kernel-trace ... bench.py`:
every slot's stream is held by k_hold until all steps are enqueued, so the trace after the last
k_hold shows the batches as the device ran them (not the tracer's per-launch host overhead).

    python bench_tools/gate_timeline.py gpurun_out/<tag>/raw/kt_kernel_trace.csv [--bin 2]
"""
import argparse
import collections
import csv
import math


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--bin", type=float, default=2.0, help="ms per timeline row")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                     r["Kernel_Name"].split("(")[0].replace("ssb::k::", "").replace("void ", "")))
    rows.sort()
    holds = [r for r in rows if r[3] == "k_hold"]
    nq = len({h[2] for h in holds})
    last = holds[-nq:]
    t0 = max(h[1] for h in last)
    win = [r for r in rows if r[0] >= min(h[0] for h in last) and r[3] != "k_hold"]
    t1 = max(r[1] for r in win)
    print("%d slot queues held; device span after release %.2f ms" % (nq, (t1 - t0) / 1e6))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in win:
        agg[r[3]][0] += 1
        agg[r[3]][1] += (r[1] - r[0]) / 1e6
    print("%-34s %5s %9s %8s" % ("kernel", "n", "busy_ms", "mean_ms"))
    for k, (n, b) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:24]:
        print("%-34s %5d %9.2f %8.3f" % (k, n, b, b / n))
    ends = collections.defaultdict(int)
    for r in win:
        ends[r[2]] = max(ends[r[2]], r[1])
    print("queue finish (ms): " + " ".join("%.1f" % ((e - t0) / 1e6) for e in sorted(ends.values())))
    # per queue (batch), the end of each stage relative to the release: what the last batches wait on
    per_q = collections.defaultdict(dict)
    for r in win:
        if r[3].startswith("__amd") or r[3].startswith("at::"):
            continue
        k = r[3].split("<")[0]
        per_q[r[2]][k] = max(per_q[r[2]].get(k, 0), r[1])
    stages = ["k_decode_count", "k_subgroup_map", "k_msm_bucket2", "k_msm_window2", "k_miller_final",
              "k_fb_rlc", "k_fb_root", "k_fb_single", "k_fb_sparse", "k_fb_level", "k_select_combine", "k_combine_sum"]
    print("per-queue stage ends (ms), by queue finish:")
    print("  " + " ".join("%9s" % s.replace("k_", "")[:9] for s in stages) + "  last")
    for q, d in sorted(per_q.items(), key=lambda kv: max(kv[1].values())):
        print("  " + " ".join("%9.2f" % ((d[s] - t0) / 1e6) if s in d else "%9s" % "-" for s in stages) +
              "  %.2f" % ((max(d.values()) - t0) / 1e6))
    step = a.bin * 1e6
    for b in range(int(math.ceil((t1 - t0) / step))):
        lo, hi = t0 + b * step, t0 + (b + 1) * step
        run = [r for r in win if r[0] < hi and r[1] > lo]
        c = collections.Counter(r[3] for r in run)
        print("%6.1f ms: %3d  %s" % (b * a.bin, len(run), ", ".join("%s x%d" % (k.replace("k_", ""), v) for k, v in c.most_common(7))))


if __name__ == "__main__":
    main()
