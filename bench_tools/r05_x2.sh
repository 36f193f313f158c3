#!/bin/bash
# round 5: two-chain lazy Fp2 products (SSB_FP2_X2 variant library) against the product library,
# interleaved: the roofline batch's subgroup / decode launches and the rate
set -o pipefail
OUT=${1:-gpurun_out/r05x2}
mkdir -p $OUT
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for i in 1 2; do
  for v in base x2; do
    if [ $v = x2 ]; then export SSB_LIB_VARIANT=x2; else unset SSB_LIB_VARIANT; fi
    for st in 20 200; do
      timeout -k 10 300 python -u bench.py $X --steps $st > $OUT/${v}_${st}_$i.json 2> $OUT/${v}_${st}_$i.err || { echo "$v failed"; tail -5 $OUT/${v}_${st}_$i.err; exit 1; }
      python -c "
import json; d=json.load(open('$OUT/${v}_${st}_$i.json')); r=d['roofline']
print('$v $st $i', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'], 'sg', r['avg_launch_ms'], r['frac'], 'dec', r['k_decode_count']['avg_launch_ms'])"
    done
  done
done
