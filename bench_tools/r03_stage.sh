#!/bin/bash
# Lane-program stage latency (bench_tools/stage_bench) and the gated per-queue timeline of the
# driver's command (bench_tools/gate_timeline.py).
#   bench_tools/r03_stage.sh TAG
set -o pipefail
TAG=${1:-r03_stage}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 60 bench_tools/stage_bench > $OUT/stage.txt 2>&1 || { echo "stage_bench failed"; cat $OUT/stage.txt; exit 1; }
cat $OUT/stage.txt
GPU_MAX_HW_QUEUES=23 SSB_DEBUG_GATE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o kt -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers > $OUT/gate.log 2>&1 || { echo "gated trace failed"; tail -20 $OUT/gate.log; exit 1; }
CSV=$(find $OUT/raw -name '*kernel_trace.csv' | head -1)
python bench_tools/gate_timeline.py "$CSV" > $OUT/gate_timeline.txt && head -45 $OUT/gate_timeline.txt
rm -rf $OUT/raw
