#!/bin/bash
# rocprofv3 kernel stats of the bench with invalid shares: bench_tools/prof_invalid.sh TAG RATE
set -o pipefail
TAG=${1:-profinv}; RATE=${2:-0.01}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --steps 12 --warmup 1 --no-cpu-baseline --invalid-rate $RATE > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
DB=$(find $OUT/prof -name '*.db' | head -1)
python bench_tools/rocpd_stats.py "$DB" > $OUT/kernel_stats.csv && cut -c1-120 $OUT/kernel_stats.csv | head -30
