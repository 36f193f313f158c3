"""Kernel statistics (rocprofv3 --stats layout: Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs) from a rocprofv3 rocpd database (run_results.db), for ROCm builds whose --stats output
is the database only.   python bench_tools/rocpd_stats.py <run_results.db> <out.csv> [grid]"""
import csv
import sqlite3
import sys


def main(db_path, out_path, by_grid=False):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, grid_x, duration from kernels").fetchall()
    agg = {}
    for name, grid, dur in rows:
        short = name.split("(")[0]
        key = (short, grid) if by_grid else short
        a = agg.setdefault(key, [0, 0, None, 0])
        a[0] += 1; a[1] += dur; a[2] = dur if a[2] is None else min(a[2], dur); a[3] = max(a[3], dur)
    total = sum(a[1] for a in agg.values()) or 1
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"] + (["Grid"] if by_grid else []))
        for key, a in sorted(agg.items(), key=lambda x: -x[1][1]):
            name = key[0] if by_grid else key
            row = [name, a[0], a[1], round(a[1] / a[0], 1), round(100.0 * a[1] / total, 2), a[2], a[3]]
            w.writerow(row + ([key[1]] if by_grid else []))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], len(sys.argv) > 3)
