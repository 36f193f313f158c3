#!/bin/bash
# collector with a separate delivery thread: GPU collector tests, then the default bench twice
set -o pipefail
OUT=${1:-gpurun_out/r04coll2}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_collector.py tests/test_collector.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/bench$i.json 2> $OUT/bench$i.err || { echo "bench $i failed"; tail -20 $OUT/bench$i.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench$i.json')); c=d['collector']
print($i, d['value'], d['value_sustained'], d['value_collector'], c.get('frac_of_value'), c.get('worker_profile_incl_warmup'), d['results_ok'])"
done
