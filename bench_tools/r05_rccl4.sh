#!/bin/bash
# round 5: RCCL at N = 1 after the spec / tail streams became three-stream-only: queue budget sweep
set -o pipefail
OUT=${1:-gpurun_out/r05rccl4}
mkdir -p $OUT
X="--steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
run() {   # name, extra args
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 1 $X --force-dist $2 > $OUT/$1.json 2> $OUT/$1.err || { echo "$1 failed"; tail -20 $OUT/$1.err; exit 1; }
  python -c "
import json
d = json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1])
print('$1', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
}
plain() {
  timeout -k 10 300 python -u bench.py --gpus 1 $X $2 > $OUT/$1.json 2> $OUT/$1.err || { echo "$1 failed"; tail -20 $OUT/$1.err; exit 1; }
  python -c "
import json
d = json.load(open('$OUT/$1.json')); print('$1', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
}
plain plain23 "" && run d23 "" && run d24 "--hw-queues 24" && run d25 "--hw-queues 25"
