#!/bin/bash
# A/B: the combine TU at one wave per SIMD (base) vs two (cw2: SSB_COMBINE_WAVES=2)
set -o pipefail
OUT=${1:-gpurun_out/r04cw2}; mkdir -p $OUT
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
SSB_LIB_VARIANT=cw2 timeout -k 10 200 python -u -m pytest tests/test_gpu_fallback.py -x -q --timeout 150 --timeout-method thread -m gpu -k "registry or pct1" > $OUT/cw2.tests.log 2>&1 || { echo "cw2 tests failed"; tail -20 $OUT/cw2.tests.log; exit 1; }
tail -1 $OUT/cw2.tests.log
for var in base cw2; do
  if [ $var = base ]; then export SSB_LIB_VARIANT=; else export SSB_LIB_VARIANT=$var; fi
  for v in "valid:" "pct1:--invalid-rate 0.01" "registry:--ids registry"; do
    name=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py $X $a > $OUT/$var.$name.json 2> $OUT/$var.$name.err || { echo "bench $var $name failed"; tail -5 $OUT/$var.$name.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$var.$name.json')); print('$var $name', d['value'], d['ms_per_step'], d['results_ok'], d['batch_latency_ms'], {k: round(v, 2) for k, v in d['kernel_ms'].items() if 'comb' in k and v > 0.1})"
  done
done
