#!/bin/bash
# fallback launches' grid cap A/B (the product build): fallback parity, then one invalid / 1e-2 / faulty operator
set -o pipefail
OUT=${1:-gpurun_out/r04grid}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -m gpu -k "fallback or invalid or committee or operator or tree or bisect" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "one:--invalid-count 1" "pct1:--invalid-rate 0.01" "badop:--bad-operator 2"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], d['batch_latency_ms'])"
done
