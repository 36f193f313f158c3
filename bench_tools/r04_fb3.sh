#!/bin/bash
# fallback launches with capped grids: bad-operator diag (hang guard), fallback parity tests, benches
set -o pipefail
OUT=${1:-gpurun_out/r04fb3}; mkdir -p $OUT
timeout -k 10 120 python -u bench_tools/diag_badop.py 4096 64 1 > $OUT/diag.log 2>&1 || { echo "diag failed"; tail -5 $OUT/diag.log; exit 1; }
tail -1 $OUT/diag.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fallback.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "one:--invalid-count 1" "pct1:--invalid-rate 0.01" "badop:--bad-operator 2" "registry:--ids registry"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], d['invalid_shares_per_batch'], d['batch_latency_ms'])"
done
bash bench_tools/r04_prof.sh $OUT "pct1:--invalid-rate 0.01"
