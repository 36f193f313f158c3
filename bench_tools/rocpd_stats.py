"""Kernel stats (name, calls, total/avg/min/max ns, percent) from a rocprofv3 rocpd SQLite db,
in the same columns as rocprofv3's --stats kernel_stats.csv.

    python bench_tools/rocpd_stats.py gpurun_out/<tag>/prof/<file>.db > profiles/<name>.csv
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), min(end - start), max(end - start) "
                     "from kernels group by name").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = []
    for name, n, s, lo, hi in sorted(rows, key=lambda r: -r[2]):
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        out.append([short, n, s, s / n, 100.0 * s / tot, lo, hi])
    return out


if __name__ == "__main__":
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in stats(sys.argv[1]):
        w.writerow([r[0], r[1], r[2], "%.1f" % r[3], "%.2f" % r[4], r[5], r[6]])
