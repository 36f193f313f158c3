#!/bin/bash
# round 6: the GPU suite, smoke(), and the driver's bench command (with the adversarial legs)
set -o pipefail
OUT=${1:-gpurun_out/r06check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -10 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -10 $OUT/bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value', 'ms_per_step', 'value_registry', 'value_invalid_1e2', 'value_bad_operator', 'value_collector', 'value_collector_wire', 'value_sustained', 'batch_latency_ms', 'value_host_buffers', 'results_ok')})
print('adv', d.get('adversarial'))
print('roofline', d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'cpu', d['cpu_baseline'])"
# the same command under rocprofv3 (kernel trace + stats; the roofline kernel's average launch must agree)
if [ "${PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof bench failed"; tail -5 $OUT/bench_prof.err; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
  head -12 $OUT/kernel_stats.csv | cut -c1-160
fi
