#!/bin/bash
# the driver's default command twice (run-to-run spread), 200 timed steps by default
set -o pipefail
OUT=${1:-gpurun_out/r04bench2}; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 600 python -u bench.py > $OUT/bench$i.json 2> $OUT/bench$i.err || { echo "bench $i failed"; tail -20 $OUT/bench$i.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench$i.json'))
print($i, {k: d.get(k) for k in ('value', 'ms_per_step', 'steps', 'value_sustained', 'value_collector', 'batch_latency_ms', 'value_host_buffers', 'results_ok')}, d['collector'].get('frac_of_value'))"
done
