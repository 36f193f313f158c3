#!/bin/bash
# round 6: G2 bucket sums in the reduced radix -- GPU suite, A/B against the engine-form MSM
# (SSB_VARIANT=msmeng, -DSSB_MSM_ENGINE) on the driver-shaped bench, alternating; then HBM counters
set -o pipefail
OUT=${1:-gpurun_out/r06k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial --steps 20"
for rep in 1 2; do
  for v in product msmeng; do
    if [ $v = product ]; then unset SSB_LIB_VARIANT; else export SSB_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u bench.py $X > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "bench $v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); r=d['roofline']; print('$v', $rep, d['value'], d['ms_per_step'], 'sus', d['value_sustained'], 'lat', d['batch_latency_ms'], 'frac', r['frac'], d['results_ok'])"
  done
done
unset SSB_LIB_VARIANT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/drv -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-registry --no-adversarial --collector-windows 0 --no-cpu-baseline > $OUT/drv.json 2> $OUT/drv.err || { echo "driver prof failed"; tail -5 $OUT/drv.err; exit 1; }
echo done
