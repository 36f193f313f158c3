#!/bin/bash
# round 5: HBM traffic counters (one group per rocprofv3 run, never with tracing) over the driver-
# shaped bench: the roofline batch (8 x C2 at depth 1) and the pipelined C2 batches, told apart by
# grid size (pmc_summary.py --by-grid)
set -o pipefail
TAG=${1:-r05pmc}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pass$i -o run -- $CMD > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pass$i.log; exit 1; }
done
python3 bench_tools/pmc_summary.py $OUT --by-grid > $OUT/summary.json && python3 -c "
import json; d=json.load(open('$OUT/summary.json'))
for k, v in sorted(d.items()):
    if any(x in k for x in ('subgroup_map', 'decode_count')):
        print(k, round(v.get('hbm_bytes_per_launch', 0)))"
