"""Per-queue device timeline of a gated run (see gate_timeline.py): for every slot queue, the
kernels of its batch with start / end in ms after the release of the gate.

    python bench_tools/queue_timeline.py gpurun_out/<tag>/raw/kt_kernel_trace.csv
"""
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                     r["Kernel_Name"].split("(")[0].replace("ssb::k::", "").replace("void ", "")))
    rows.sort()
    holds = [r for r in rows if r[3] == "k_hold"]
    nq = len({h[2] for h in holds})
    last = holds[-nq:]
    t0 = max(h[1] for h in last)
    win = [r for r in rows if r[0] >= min(h[0] for h in last) and r[3] != "k_hold"]
    byq = {}
    for r in win:
        byq.setdefault(r[2], []).append(r)
    for q, rs in sorted(byq.items(), key=lambda kv: kv[1][-1][1]):
        print("queue %d  end %.2f" % (q, (rs[-1][1] - t0) / 1e6))
        print("   " + "  ".join("%s %.1f-%.1f" % (r[3][:14], (r[0] - t0) / 1e6, (r[1] - t0) / 1e6)
                                for r in rs if (r[1] - r[0]) > 20000))


if __name__ == "__main__":
    main()
