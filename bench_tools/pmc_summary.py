"""Summarise rocprofv3 --pmc counter_collection.csv files (bench_tools/pmc.sh) per kernel:
average counter value per dispatch; HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half of
wide coalesced reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, FETCH/WRITE_SIZE in KB.

    python bench_tools/pmc_summary.py gpurun_out/<tag> [--by-grid] > summary.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("ssb::k::", "")


def main(root, by_grid=False):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row.get("Kernel_Name", ""))
                if by_grid:   # one entry per launch shape (e.g. the roofline batch vs the C2 batches)
                    gs = [v for c, v in row.items() if c and c.startswith("Grid_Size")]
                    k = "%s@%s" % (k, "x".join(gs))
                c = row.get("Counter_Name", "")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                vals[k][c].append(v)
    out = {}
    for k, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in d or "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = 2 * 1024 * d.get("FETCH_SIZE", 0.0) + 1024 * d.get("WRITE_SIZE", 0.0)
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"]:
            d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        if "SQ_ACTIVE_INST_VALU" in d and "SQ_BUSY_CYCLES" in d and d["SQ_BUSY_CYCLES"]:
            d["valu_active_per_busy_cycle"] = d["SQ_ACTIVE_INST_VALU"] / d["SQ_BUSY_CYCLES"]
        out[k] = d
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], by_grid="--by-grid" in sys.argv)
