#!/bin/bash
# round 6 (closing): the MSM latency forms at every pipeline depth (SSB_MSM_LAT=a) against the default
# (one slot only), the driver's 20-step command without the side legs, alternating
set -o pipefail
OUT=${1:-gpurun_out/r06lat}
mkdir -p $OUT
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial"
for rep in 1 2 3; do
  for v in default all; do
    if [ $v = all ]; then export SSB_MSM_LAT=a; else unset SSB_MSM_LAT; fi
    timeout -k 10 300 python -u bench.py $X --steps 20 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "bench $v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v', $rep, d['value'], d['ms_per_step'], 'sus', d['value_sustained'], 'lat', d['batch_latency_ms'], d['results_ok'])"
  done
done
unset SSB_MSM_LAT
