#!/bin/bash
# round 5: the lane-uniform ratio combine (phases in the terms / sum launches), the wire-record
# collector, the context lock -- GPU tests of those paths, then the rate at the driver's 20 steps,
# seq vs registry vs registry through the general combine (SSB_NO_RATIO), invalid patterns, and the
# default bench line
set -o pipefail
OUT=${1:-gpurun_out/r05reg}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_collector.py -x -v --timeout 150 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for v in "seq20:--steps 20" "reg20:--steps 20 --ids registry" "reg200:--steps 200 --ids registry" "regnr20:--steps 20 --ids registry" "one20:--steps 20 --invalid-count 1" "badop20:--steps 20 --bad-operator 1" "pct20:--steps 20 --invalid-rate 0.01"; do
  name=${v%%:*}; a=${v#*:}
  if [ "$name" = regnr20 ]; then export SSB_NO_RATIO=1; else unset SSB_NO_RATIO; fi
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
done
unset SSB_NO_RATIO
timeout -k 10 600 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/default20.json 2> $OUT/default20.err || { echo "bench default failed"; tail -5 $OUT/default20.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/default20.json'))
print({k: d.get(k) for k in ('value', 'ms_per_step', 'value_registry', 'value_sustained', 'value_collector', 'batch_latency_ms', 'value_host_buffers', 'results_ok')})
print('registry', d.get('registry'))"
