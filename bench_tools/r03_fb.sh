#!/bin/bash
# Fallback iteration: the -m gpu tests, C2 all-valid / 1 invalid / 1e-2 and C4 1e-2 at the driver's
# settings, then the gated per-queue timeline of the one-invalid run.
#   bench_tools/r03_fb.sh TAG
set -o pipefail
TAG=${1:-r03fb}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { echo "$nm failed"; tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$nm.json'));print('$nm', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['kernel_ms']['k_fallback_verify'], d['invalid_shares_per_batch'], d['results_ok'])"
}
run c2_valid
run c2_one --invalid-count 1
run c2_1e2 --invalid-rate 1e-2
run c4_1e2 --config C4_per_gpu --invalid-rate 1e-2
bench_tools/r03_one.sh ${TAG}_one
