#!/bin/bash
# Interleaved A/B of the driver's bench command: the product library vs an experiment build
# (safestakeoperator_amd/libssbls_<VARIANT>.so, SSB_VARIANT=<VARIANT> SSB_VARIANT_DEFS=... build).
#   bench_tools/r03_ab.sh TAG VARIANT [PAIRS]
set -o pipefail
TAG=$1; VAR=$2; K=${3:-3}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $K); do
  for v in base $VAR; do
    if [ $v = base ]; then envs="SSB_X=0"; else envs="SSB_LIB_VARIANT=$v"; fi
    env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers > $OUT/$v$i.json 2> $OUT/$v$i.err || { echo "$v $i FAILED"; tail -5 $OUT/$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v', $i, d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
  done
done
