#!/bin/bash
# A/B of a build: the GPU parity tests, C2 at the driver's settings (twice), 1 and 2 invalid shares
# per batch, then the gated timeline of the all-valid run.
#   bench_tools/r03_ab2.sh TAG
set -o pipefail
TAG=${1:-r03ab2}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for a in "v1" "v2" "one --invalid-count 1" "two --invalid-count 2" "e2 --invalid-rate 1e-2"; do
  set -- $a; nm=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { echo "$nm failed"; tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$nm.json'));print('$nm', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['kernel_ms']['k_miller'], d['kernel_ms']['k_fallback_verify'], d['results_ok'])"
done
GPU_MAX_HW_QUEUES=23 SSB_DEBUG_GATE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o kt -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers > $OUT/gate.log 2>&1 || { echo "gated trace failed"; tail -20 $OUT/gate.log; exit 1; }
CSV=$(find $OUT/raw -name '*kernel_trace.csv' | head -1)
python bench_tools/gate_timeline.py "$CSV" > $OUT/gate_timeline.txt && head -40 $OUT/gate_timeline.txt
rm -rf $OUT/raw
