#!/bin/bash
# NAF digit chains (value form): a short guarded run first, then parity and the registry benches
set -o pipefail
OUT=${1:-gpurun_out/r04naf}; mkdir -p $OUT
SSB_LIB_VARIANT=naf timeout -k 10 90 python -u bench.py --steps 2 --warmup 1 --pipeline 1 --ids registry --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 > $OUT/guard.json 2> $OUT/guard.err || { echo "guard failed rc $?"; tail -3 $OUT/guard.err; exit 1; }
echo guard ok
SSB_LIB_VARIANT=naf timeout -k 10 400 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "pct1:--invalid-rate 0.01" "registry:--ids registry" "registry_one:--ids registry --invalid-count 1"; do
  name=${v%%:*}; a=${v#*:}
  SSB_LIB_VARIANT=naf timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], d['batch_latency_ms'])"
done
