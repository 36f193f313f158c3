#!/bin/bash
# round 6 (closing): the group tests' bucket mode (SSB_FB_BUCKET=1: one RLC check per operator-id
# bucket across the roots) -- fallback / C2 parity tests in that mode, then the driver-shaped bench
# (adversarial legs on, no collector / registry / sustained) alternating default and bucket mode
set -o pipefail
OUT=${1:-gpurun_out/r06bk}
mkdir -p $OUT
export TMPDIR=/tmp
SSB_FB_BUCKET=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --steps 20"
for rep in 1 2; do
  for v in default bucket; do
    if [ $v = bucket ]; then export SSB_FB_BUCKET=1; else unset SSB_FB_BUCKET; fi
    timeout -k 10 300 python -u bench.py $X > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "bench $v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); a=d['adversarial']; print('$v', $rep, d['value'], 'bad_op', d['value_bad_operator'], a['bad_operator']['frac_of_value'], a['bad_operator']['results_ok'], 'pct1', d['value_invalid_1e2'], a['invalid_1e2']['results_ok'], d['results_ok'])"
  done
done
unset SSB_FB_BUCKET
