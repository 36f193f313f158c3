#!/bin/bash
# round 6 (closing): FETCH / WRITE counters of the driver-shaped bench (no side legs) with the
# XCD-owned scatter (default) and the former per-block scatter (SSB_SCATTER_XCD=0)
set -o pipefail
OUT=${1:-gpurun_out/r06scp}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --no-adversarial"
for v in owned old; do
  if [ $v = old ]; then export SSB_SCATTER_XCD=0; else unset SSB_SCATTER_XCD; fi
  mkdir -p $OUT/$v
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    echo "[pmc] $v pass $i: $grp"
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/$v/pass$i -o run -- $CMD > $OUT/$v/pass$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/$v/pass$i.log; exit 1; }
  done
  python3 bench_tools/pmc_summary.py $OUT/$v --by-grid > $OUT/$v/summary.json && python3 -c "
import json; d=json.load(open('$OUT/$v/summary.json'))
for k, v in sorted(d.items()):
    if any(x in k for x in ('subgroup_map', 'decode_count', 'msm_bucket2')):
        print('$v', k, {c: round(x, 1) for c, x in v.items() if c in ('hbm_bytes_per_launch', 'FETCH_SIZE', 'WRITE_SIZE')})"
done
unset SSB_SCATTER_XCD
