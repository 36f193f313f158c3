#!/bin/bash
# round 5: slot stream priorities (SSB_SLOT_PRIO=1: three bands) against none, interleaved, at the
# driver's 20 steps and over 200
set -o pipefail
OUT=${1:-gpurun_out/r05prio}
mkdir -p $OUT
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for i in 1 2; do
  for v in "base" "prio"; do
    if [ $v = prio ]; then export SSB_SLOT_PRIO=1; else unset SSB_SLOT_PRIO; fi
    for st in 20 200; do
      timeout -k 10 300 python -u bench.py $X --steps $st > $OUT/${v}_${st}_$i.json 2> $OUT/${v}_${st}_$i.err || { echo "$v failed"; tail -5 $OUT/${v}_${st}_$i.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${v}_${st}_$i.json')); print('$v $st $i', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
    done
  done
done
