#!/bin/bash
# Adversarial throughput (BASELINE C4's invalid rates) in the bench's 20-slot one-stream
# configuration: the driver's command with 1 invalid share per batch, 1e-4 (rounded up: >= 1 per
# C2 batch) and 1e-2, for C2 and C4_per_gpu; then kernel stats of the 1% C2 run.
#   bench_tools/r03_invalid.sh TAG
set -o pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { echo "$nm failed"; tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$nm.json'));print('$nm', d['value'], d['ms_per_step'], d['invalid_shares_per_batch'], d['results_ok'])"
}
run c2_valid
run c2_one --invalid-count 1
run c2_1e4 --invalid-count 2
run c2_1e2 --invalid-rate 1e-2
run c4_valid --config C4_per_gpu
run c4_1e4 --config C4_per_gpu --invalid-rate 1e-4
run c4_1e2 --config C4_per_gpu --invalid-rate 1e-2
GPU_MAX_HW_QUEUES=23 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --invalid-rate 1e-2 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
DB=$(find $OUT/prof -name '*.db' | head -1)
python bench_tools/rocpd_stats.py "$DB" > $OUT/kernel_stats_1e2.csv && cut -c1-110 $OUT/kernel_stats_1e2.csv | head -20
rm -rf $OUT/prof
