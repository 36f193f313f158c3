#!/bin/bash
# round 6: A/B of the MSM bucket sums (G2 and G1) in the reduced radix (SSB_VARIANT=msmr28,
# -DSSB_MSM_R28) against the product's engine-form buckets, alternating; the variant's GPU MSM tests
set -o pipefail
OUT=${1:-gpurun_out/r06q}
mkdir -p $OUT
export TMPDIR=/tmp
SSB_LIB_VARIANT=msmr28 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests_msmr28.log 2>&1 || { echo "variant gpu tests failed"; tail -30 $OUT/gpu_tests_msmr28.log; exit 1; }
tail -1 $OUT/gpu_tests_msmr28.log
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial --steps 20"
for rep in 1 2; do
  for v in product msmr28; do
    if [ $v = product ]; then unset SSB_LIB_VARIANT; else export SSB_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u bench.py $X > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "bench $v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v', $rep, d['value'], d['ms_per_step'], 'sus', d['value_sustained'], 'lat', d['batch_latency_ms'], d['results_ok'])"
  done
done
