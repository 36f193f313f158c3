#!/bin/bash
# smoke(), then the driver's command (20 steps) at several pipeline depths.
#   bench_tools/r03_depth.sh TAG "10 14 16 20"
set -o pipefail
TAG=${1:-r03depth}; DEPTHS=${2:-"10 14 16 20"}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for d in $DEPTHS; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --pipeline $d > $OUT/d$d.json 2> $OUT/d$d.err || { tail -20 $OUT/d$d.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/d$d.json'));print($d, d['value'], d['ms_per_step'], d.get('batch_latency_ms'))"
done
