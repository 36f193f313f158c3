#!/bin/bash
# registry ids through the general combine with unit_lagrange_fast: parity, then the benches (200 steps)
set -o pipefail
OUT=${1:-gpurun_out/r04lagfast}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "pct1:--invalid-rate 0.01" "registry:--ids registry" "registry_one:--ids registry --invalid-count 1"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], d['batch_latency_ms'])"
done
