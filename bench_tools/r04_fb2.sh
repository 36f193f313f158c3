#!/bin/bash
# round 4: committee stage (exclusion + singles, group tests + deduction) and registry ids:
# parity tests, then the driver's C2 command at each invalid pattern / id scheme, and a kernel
# profile of the 1e-2 run
set -o pipefail
OUT=${1:-gpurun_out/r04fb2}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_collector.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "one:--invalid-count 1" "pct1:--invalid-rate 0.01" "badop:--bad-operator 2" "registry:--ids registry" "registry_one:--ids registry --invalid-count 1"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], d['invalid_shares_per_batch'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pct1 -o run -- python -u bench.py $X --invalid-rate 0.01 > $OUT/prof_pct1.json 2> $OUT/prof_pct1.err || { echo "prof failed"; tail -5 $OUT/prof_pct1.err; exit 1; }
f=$(find $OUT/prof_pct1 -name "*kernel_stats.csv" | head -1); cp $f $OUT/pct1_kernel_stats.csv; head -16 $OUT/pct1_kernel_stats.csv | cut -c1-160
