#!/bin/bash
# round 4: registry ids (ratio combine) parity + rate, and a kernel profile of the 1e-2 run
set -o pipefail
OUT=${1:-gpurun_out/r04reg}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fallback.py -x -v --timeout 200 --timeout-method thread -m gpu -k "registry or one" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "seq:" "registry:--ids registry" "registry_noratio:--ids registry"; do
  name=${v%%:*}; a=${v#*:}
  if [ "$name" = registry_noratio ]; then export SSB_NO_RATIO=1; fi
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'])"
done
unset SSB_NO_RATIO
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_pct1 -o run -- python -u bench.py $X --invalid-rate 0.01 > $OUT/prof_pct1.json 2> $OUT/prof_pct1.err || { echo "prof failed"; tail -5 $OUT/prof_pct1.err; exit 1; }
find $OUT/prof_pct1 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/pct1_kernel_stats.csv
head -20 $OUT/pct1_kernel_stats.csv
