#!/bin/bash
# the roofline launch in the kernel trace: bench.py (short) under rocprofv3 --kernel-trace --stats,
# k_subgroup_map / k_decode_count durations per grid size (the 8 x C2 roofline batch has its own grid)
set -o pipefail
OUT=${1:-gpurun_out/r04roof}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "prof failed"; tail -5 $OUT/bench.err; exit 1; }
kt=$(find $OUT/prof -name "*kernel_trace.csv" | head -1); st=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp $st $OUT/roof_kernel_stats.csv
python3 - "$kt" "$OUT/roofline_launches.json" "$OUT/bench.json" <<'PY'
import csv, json, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(list)
for r in rows:
    n = r.get("Kernel_Name", "")
    if "k_subgroup_map" in n or "k_decode_count" in n:
        g = "x".join(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z") if k in r) or r.get("Grid_Size", "")
        agg[("k_subgroup_map" if "subgroup" in n else "k_decode_count") + "@" + g].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
b = json.load(open(sys.argv[3]))
out = {k: {"launches": len(v), "avg_ms": round(sum(v) / len(v), 4), "min_ms": round(min(v), 4), "max_ms": round(max(v), 4)} for k, v in sorted(agg.items())}
out["_bench_roofline"] = {k: b["roofline"].get(k) for k in ("avg_launch_ms", "achieved", "frac", "timing")}
json.dump(out, open(sys.argv[2], "w"), indent=1)
for k, v in out.items(): print(k, v)
PY
find $OUT/prof -name "*.csv" -delete
