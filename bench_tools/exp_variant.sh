#!/bin/bash
# Compare library variants (one GPU call): bench_tools/exp_variant.sh TAG "variant1 variant2" "depths"
# ("base" = libssbls.so).  Each variant: GPU parity tests, then the bench at every depth.
set -o pipefail
TAG=${1:-var}; VARS=${2:-base}; DEPTHS=${3:-12}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in $VARS; do
  if [ "$v" = base ]; then export SSB_LIB_VARIANT=; else export SSB_LIB_VARIANT=$v; fi
  if [ -n "$TESTS" ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/$v.tests.log 2>&1 || { echo "$v tests failed"; tail -30 $OUT/$v.tests.log; exit 1; }
    echo "$v: $(tail -1 $OUT/$v.tests.log)"
  fi
  for d in $DEPTHS; do
    timeout -k 10 240 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline --pipeline $d > $OUT/$v.d$d.json 2> $OUT/$v.d$d.err || { tail -20 $OUT/$v.d$d.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v.d$d.json'));print('$v', $d, d['value'], d['ms_per_step'], d.get('batch_latency_ms'), {k:round(v,3) for k,v in d['kernel_ms'].items() if v>0.05})"
  done
done
