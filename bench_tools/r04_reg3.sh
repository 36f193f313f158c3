#!/bin/bash
# interleaved [M^-1] T on one lane + one round of suspect checks: registry / fallback parity, benches
set -o pipefail
OUT=${1:-gpurun_out/r04reg3}; mkdir -p $OUT
X="--steps 2 --warmup 1 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --pipeline 1"
timeout -k 10 90 python -u bench.py $X --ids registry > $OUT/guard.json 2> $OUT/guard.err || { echo "guard failed"; tail -5 $OUT/guard.err; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_fallback.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "one:--invalid-count 1" "pct1:--invalid-rate 0.01" "registry:--ids registry" "registry_one:--ids registry --invalid-count 1"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], d['invalid_shares_per_batch'], d['batch_latency_ms'], {k: round(v, 2) for k, v in d['kernel_ms'].items() if v > 0.3})"
done
