#!/bin/bash
# One GPU call: parity tests, bench, rocprofv3 kernel stats.
#   bench_tools/gpu_check.sh TAG [STEPS] [notests]
set -o pipefail
TAG=${1:-run}; STEPS=${2:-10}; MODE=${3:-all}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" != "notests" ]; then
  echo "[gpu_check] tests"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
echo "[gpu_check] bench"
timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "[gpu_check] rocprof"
GPU_MAX_HW_QUEUES=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
DB=$(find $OUT/prof -name '*.db' | head -1)
python bench_tools/rocpd_stats.py "$DB" > $OUT/kernel_stats.csv && cut -c1-110 $OUT/kernel_stats.csv | head -24
