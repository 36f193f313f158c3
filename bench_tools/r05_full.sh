#!/bin/bash
# round 5: the whole GPU suite, the input patterns at the driver's 20 steps, the default bench line,
# and the RCCL path at N = 1 (torchrun, one rank) beside it
set -o pipefail
OUT=${1:-gpurun_out/r05full}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for v in "seq20:--steps 20" "reg20:--steps 20 --ids registry" "one20:--steps 20 --invalid-count 1" "badop20:--steps 20 --bad-operator 1" "pct20:--steps 20 --invalid-rate 0.01"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/default20.json 2> $OUT/default20.err || { echo "bench default failed"; tail -5 $OUT/default20.err; exit 1; }
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --force-dist > $OUT/n1_rccl.json 2> $OUT/n1_rccl.err || { echo "rccl n1 failed"; tail -20 $OUT/n1_rccl.err; exit 1; }
python -c "
import json
for n in ('default20', 'n1_rccl'):
    d = json.loads(open('$OUT/%s.json' % n).read().strip().splitlines()[-1])
    print(n, {k: d.get(k) for k in ('value', 'ms_per_step', 'value_registry', 'value_collector', 'value_collector_wire', 'value_sustained', 'batch_latency_ms', 'results_ok')})
    print('  roofline', d.get('roofline'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
