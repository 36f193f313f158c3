"""Per-kernel summary of a rocprofv3 kernel-trace database (run_results.db): calls, total and
average duration, grid, scratch -- optionally only dispatches of a given grid size.
    python bench_tools/prof_db.py DB [DB2]    (two: side by side, the second's delta)"""
import sqlite3
import sys
import re


def summary(db):
    con = sqlite3.connect(db)
    out = {}
    for name, n, tot, grid, scr in con.execute(
            "select name, count(*), sum(duration), max(grid_x), max(scratch_size) from kernels group by name"):
        short = re.sub(r"\(.*", "", name).split("::")[-1]
        o = out.setdefault(short, [0, 0, 0, 0])
        o[0] += n; o[1] += tot; o[2] = max(o[2], grid); o[3] = max(o[3], scr or 0)
    span = con.execute("select min(start), max(end) from kernels").fetchone()
    return out, (span[1] - span[0]) / 1e6


def main():
    dbs = sys.argv[1:]
    res = [summary(d) for d in dbs]
    names = sorted(set().union(*[r[0].keys() for r in res]), key=lambda k: -max(r[0].get(k, [0, 0])[1] for r in res))
    print("%-28s" % "kernel" + "".join("%10s %9s %9s %7s |" % ("calls", "tot_ms", "avg_us", "scr") for _ in res))
    for k in names:
        row = "%-28s" % k[:28]
        for r in res:
            v = r[0].get(k)
            row += ("%10d %9.2f %9.1f %7d |" % (v[0], v[1] / 1e6, v[1] / v[0] / 1e3, v[3])) if v else " " * 39 + "|"
        print(row)
    print("span_ms", [round(r[1], 1) for r in res])


if __name__ == "__main__":
    main()
