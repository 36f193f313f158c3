#!/bin/bash
# Throughput with invalid shares (one GPU call): bench_tools/exp_invalid.sh TAG "0.0001 0.01"
set -o pipefail
TAG=${1:-inv}; RATES=${2:-"0.0001 0.01"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $RATES; do
  timeout -k 10 300 python -u bench.py --steps 24 --warmup 2 --no-cpu-baseline --invalid-rate $r > $OUT/r$r.json 2> $OUT/r$r.err || { tail -20 $OUT/r$r.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r$r.json'));print('$r', d['value'], d['ms_per_step'], d['results_ok'], d['invalid_shares_per_batch'], d.get('batch_latency_ms'), d['kernel_ms']['k_fallback_verify'])"
done
