#!/bin/bash
# Gated per-queue timeline of the driver's command with ONE invalid share per batch (every batch runs
# the exact fallback): where the adversarial case's time goes.
#   bench_tools/r03_one.sh TAG
set -o pipefail
TAG=${1:-r03_one}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=23 SSB_DEBUG_GATE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o kt -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --invalid-count 1 > $OUT/gate.log 2>&1 || { echo "gated trace failed"; tail -20 $OUT/gate.log; exit 1; }
CSV=$(find $OUT/raw -name '*kernel_trace.csv' | head -1)
python bench_tools/gate_timeline.py "$CSV" > $OUT/gate_timeline.txt && head -45 $OUT/gate_timeline.txt
rm -rf $OUT/raw
