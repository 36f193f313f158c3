#!/bin/bash
# round 4 full check: every -m gpu test, smoke, then the driver's default bench command
set -o pipefail
OUT=${1:-gpurun_out/r04full}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print({k: d.get(k) for k in ('value', 'ms_per_step', 'value_sustained', 'value_collector', 'batch_latency_ms', 'value_host_buffers', 'results_ok')})
print('collector', {k: v for k, v in d.get('collector', {}).items() if k != 'worker_profile'})
print('roofline', {k: d['roofline'].get(k) for k in ('achieved', 'frac', 'traffic', 'avg_launch_ms')})
print('cpu', d.get('cpu_baseline'))"
