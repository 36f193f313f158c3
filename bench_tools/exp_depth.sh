#!/bin/bash
# Throughput vs pipeline depth (one GPU call): bench_tools/exp_depth.sh TAG "8 12 16"
set -o pipefail
TAG=${1:-depth}; DEPTHS=${2:-"8 12 16"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for d in $DEPTHS; do
  timeout -k 10 240 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline --pipeline $d $EXTRA > $OUT/d$d.json 2> $OUT/d$d.err || { tail -20 $OUT/d$d.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/d$d.json'));print($d, d['value'], d['ms_per_step'], d.get('batch_latency_ms'))"
done
