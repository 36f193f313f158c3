#!/bin/bash
# Pipeline depth x hash streams x tail streams sweep at the driver's step count (one GPU call).
#   bench_tools/exp_streams.sh TAG "depth:hash:tails:g1" ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for cfg in "$@"; do
  IFS=: read d h tl g <<< "$cfg"
  g=${g:-0}
  SSB_HASH_STREAMS=$h SSB_TAILS=$tl SSB_G1_STREAMS=$g timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --pipeline $d --no-cpu-baseline \
    > $OUT/$d-$h-$tl-$g.json 2> $OUT/$d-$h-$tl-$g.err || { tail -5 $OUT/$d-$h-$tl-$g.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$d-$h-$tl-$g.json'));print('$cfg', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
done
