#!/bin/bash
# round 5: exclusion quarters paired on their own blocks -- fallback parity tests, traces, patterns
set -o pipefail
OUT=${1:-gpurun_out/r05fb3}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for p in one pct; do
  SSB_LIB_VARIANT=trace timeout -k 10 200 python -u bench_tools/trace_fb.py $p > $OUT/trace_$p.txt 2>&1 || { echo "trace $p failed"; tail -5 $OUT/trace_$p.txt; exit 1; }
  grep -v "^W\|amdgpu.ids" $OUT/trace_$p.txt
done
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for v in "one20:--steps 20 --invalid-count 1" "pct20:--steps 20 --invalid-rate 0.01" "seq20:--steps 20"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
done
