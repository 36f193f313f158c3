#!/bin/bash
# round 4 final: every -m gpu test, smoke, the driver's default bench command, and its kernel profile
set -o pipefail
OUT=${1:-gpurun_out/r04final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print({k: d.get(k) for k in ('value', 'ms_per_step', 'value_sustained', 'value_collector', 'batch_latency_ms', 'value_host_buffers', 'results_ok')})
print('roofline', {k: d['roofline'].get(k) for k in ('achieved', 'frac', 'traffic', 'avg_launch_ms')})"
timeout -k 10 500 python -u bench.py --gpus 2 --dist-backend gloo > $OUT/gloo2.json 2> $OUT/gloo2.err || { echo "gloo2 failed"; tail -20 $OUT/gloo2.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/gloo2.json'))
print('gloo2', {k: d.get(k) for k in ('n_gpus', 'value', 'ms_per_step', 'value_sustained', 'value_collector', 'results_ok')})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "prof failed"; tail -5 $OUT/prof_bench.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/final_kernel_stats.csv
find $OUT/prof -name "*.csv" ! -name "*kernel_stats.csv" -delete
head -12 $OUT/final_kernel_stats.csv | cut -c1-150
