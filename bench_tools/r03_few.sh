#!/bin/bash
# The few-invalid parity tests, then C2 at 1 and 2 invalid shares per batch (driver settings).
#   bench_tools/r03_few.sh TAG
set -o pipefail
TAG=${1:-r03few}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k "few_invalid or fallback" --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for a in "c2_one --invalid-count 1" "c2_two --invalid-count 2" "c2_three --invalid-count 3"; do
  set -- $a; nm=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { echo "$nm failed"; tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$nm.json'));print('$nm', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['kernel_ms']['k_fallback_verify'], d['invalid_shares_per_batch'], d['results_ok'])"
done
