#!/bin/bash
# round 6: the square roots' powers with the reduced-radix squaring -- GPU suite, then the
# driver-shaped bench twice (20 steps + 1,000 sustained)
set -o pipefail
OUT=${1:-gpurun_out/r06o}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial --steps 20"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $X > $OUT/b$rep.json 2> $OUT/b$rep.err || { echo "bench $rep failed"; tail -5 $OUT/b$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b$rep.json')); r=d['roofline']; print('b', $rep, d['value'], d['ms_per_step'], 'sus', d['value_sustained'], 'lat', d['batch_latency_ms'], 'frac', r['frac'], 'dec_ms', r['k_decode_count']['avg_launch_ms'], d['results_ok'])"
done
