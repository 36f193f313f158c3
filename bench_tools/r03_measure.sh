#!/bin/bash
# One GPU call: the driver's bench command three times (the first with the CPU baseline), then the
# gated kernel-trace timeline of the 20-step run (bench_tools/gate_timeline.py) and its kernel stats.
#   bench_tools/r03_measure.sh TAG [extra bench args...]
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  extra=""; [ $i -gt 1 ] && extra="--no-cpu-baseline"
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 $extra "$@" > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench $i failed"; tail -20 $OUT/b$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$i.json'));print('bench $i', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['value_host_buffers'], d['results_ok'])"
done
GPU_MAX_HW_QUEUES=23 SSB_DEBUG_GATE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o kt -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers "$@" > $OUT/gate.log 2>&1 || { echo "gated trace failed"; tail -20 $OUT/gate.log; exit 1; }
CSV=$(find $OUT/raw -name '*kernel_trace.csv' | head -1)
python bench_tools/gate_timeline.py "$CSV" > $OUT/gate_timeline.txt && head -24 $OUT/gate_timeline.txt
rm -rf $OUT/raw
