#!/bin/bash
# round 6: A/B of the reduced radix -- product library (r28 subgroup check and square-root powers)
# against the engine's 12 x 32-bit form for both (experiment build SSB_VARIANT=eng, SSB_VARIANT_DEFS=
# "-DSSB_SG_ENGINE -DSSB_POW_ENGINE") and for the subgroup check only (sg32, first pass), the driver's
# 20-step command without the side legs, alternating; roofline (k_subgroup_map at 8 x C2) from each
set -o pipefail
OUT=${1:-gpurun_out/r06ab}
mkdir -p $OUT
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial"
for rep in 1 2; do
  VS="product eng"
  for v in $VS; do
    if [ $v = product ]; then unset SSB_LIB_VARIANT; else export SSB_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u bench.py $X --steps 20 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "bench $v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); r=d['roofline']; print('$v', $rep, d['value'], d['ms_per_step'], 'sus', d['value_sustained'], 'lat', d['batch_latency_ms'], 'sg_ms', r['avg_launch_ms'], 'frac', r['frac'], 'dec_ms', r['k_decode_count']['avg_launch_ms'], d['results_ok'])"
  done
done
unset SSB_LIB_VARIANT
