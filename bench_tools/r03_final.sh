#!/bin/bash
# Round-3 final evidence in one GPU call: tests + the driver's command x3 + gated timeline
# (r03_check_measure.sh), the rocprofv3 kernel stats of the driver's command, the adversarial
# runs (r03_invalid.sh) and the one-invalid gated timeline (r03_one.sh).
#   bench_tools/r03_final.sh TAG
set -o pipefail
TAG=${1:-r03final}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bench_tools/r03_check_measure.sh $TAG || exit 1
GPU_MAX_HW_QUEUES=23 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.log || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
DB=$(find $OUT/prof -name '*.db' | head -1)
python bench_tools/rocpd_stats.py "$DB" > $OUT/kernel_stats.csv && cut -c1-110 $OUT/kernel_stats.csv | head -12
rm -rf $OUT/prof
bench_tools/r03_invalid.sh ${TAG}_inv && bench_tools/r03_one.sh ${TAG}_one
