#!/bin/bash
# round 5: exclusion check with X cut into parts and per-root products; group tests in a scattered
# item order with lane-program quarter combines -- fallback parity tests, the fallback patterns, then
# the traces (experiment build)
set -o pipefail
OUT=${1:-gpurun_out/r05xp}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for v in "pct20:--steps 20 --invalid-rate 0.01" "one20:--steps 20 --invalid-count 1" "badop20:--steps 20 --bad-operator 1" "seq20:--steps 20"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
done
for p in one pct badop; do
  SSB_LIB_VARIANT=trace timeout -k 10 150 python -u bench_tools/trace_fb.py $p > $OUT/trace_$p.txt 2>&1 || { echo "trace $p failed"; tail -5 $OUT/trace_$p.txt; exit 1; }
  grep -v "^W\|amdgpu.ids" $OUT/trace_$p.txt
done
