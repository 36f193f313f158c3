#!/bin/bash
# round 5: the sqrt table in registers (fp_pow_sw_inl) -- decode launch time / traffic and the rate
set -o pipefail
OUT=${1:-gpurun_out/r05dec}
mkdir -p $OUT
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $X --steps 20 > $OUT/s20_$i.json 2> $OUT/s20_$i.err || { echo "bench failed"; tail -5 $OUT/s20_$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py $X --steps 200 > $OUT/s200_$i.json 2> $OUT/s200_$i.err || { echo "bench failed"; tail -5 $OUT/s200_$i.err; exit 1; }
  python -c "
import json
for n in ('s20_$i', 's200_$i'):
    d = json.load(open('$OUT/%s.json' % n)); r = d['roofline']
    print(n, d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'], 'dec', r['k_decode_count']['avg_launch_ms'], r['k_decode_count']['frac'], 'sg', r['avg_launch_ms'], 'kms', d['kernel_ms'].get('k_decode'), d['kernel_ms'].get('k_hash_to_g2'))"
done
