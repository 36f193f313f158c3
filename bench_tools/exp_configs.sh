#!/bin/bash
# The BASELINE.json configs other than the headline, one bench line each (one GPU call):
#   bench_tools/exp_configs.sh TAG "C3_3of4 C3_5of7 C4_per_gpu C5_per_gpu"
set -o pipefail
TAG=${1:-configs}; CFGS=${2:-"C3_3of4 C3_5of7 C4_per_gpu C5_per_gpu"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for c in $CFGS; do
  echo "[exp_configs] $c $(date +%T)"
  timeout -k 10 400 python -u bench.py --config $c --steps 6 --warmup 1 --no-cpu-baseline --no-host-buffers > $OUT/$c.json 2> $OUT/$c.err || { tail -20 $OUT/$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', d['value'], d['combined_sigs_per_s'], d['ms_per_step'], d['results_ok'], d['batch_latency_ms'], d['step_roofline']['frac'])"
done
