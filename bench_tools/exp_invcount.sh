#!/bin/bash
# Throughput with exactly C invalid shares per C2 batch (one GPU call): bench_tools/exp_invcount.sh TAG "1 2 4"
set -o pipefail
TAG=${1:-invc}; COUNTS=${2:-"1 2 4"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for c in $COUNTS; do
  timeout -k 10 300 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline --invalid-count $c > $OUT/c$c.json 2> $OUT/c$c.err || { tail -20 $OUT/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c$c.json'));print('$c', d['value'], d['ms_per_step'], d['results_ok'], d['invalid_shares_per_batch'], d.get('batch_latency_ms'), d['kernel_ms']['k_fallback_verify'])"
done
