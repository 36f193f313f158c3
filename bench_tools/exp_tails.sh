#!/bin/bash
# Invalid-share throughput vs the number of tail streams (one GPU call):
#   bench_tools/exp_tails.sh TAG "1 2 4" "0 0.01"
set -o pipefail
TAG=${1:-tails}; TAILS=${2:-"1 2 4"}; RATES=${3:-"0 0.01"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for k in $TAILS; do
  for r in $RATES; do
    SSB_TAILS=$k timeout -k 10 300 python -u bench.py --steps 24 --warmup 2 --no-cpu-baseline --invalid-rate $r > $OUT/t$k-r$r.json 2> $OUT/t$k-r$r.err || { tail -20 $OUT/t$k-r$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/t$k-r$r.json'));print('tails $k rate $r', d['value'], d['ms_per_step'], d['results_ok'], d['invalid_shares_per_batch'], d.get('batch_latency_ms'), d['kernel_ms']['k_fallback_verify'])"
  done
done
