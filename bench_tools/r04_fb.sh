#!/bin/bash
# round 4: the committee stage of the fallback -- parity tests, then the driver's C2 command at
# one invalid share per batch, 1% invalid, a bad operator, and all-valid (bench_tools/r04_fb.sh OUT)
set -o pipefail
OUT=${1:-gpurun_out/r04fb}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_collector.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "one:--invalid-count 1" "pct1:--invalid-rate 0.01" "badop:--bad-operator 2"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], d['invalid_shares_per_batch'])"
done
