#!/bin/bash
# round 5: RCCL at N = 1 (torchrun, one rank, --force-dist) against the hardware-queue budget:
# which GPU_MAX_HW_QUEUES leaves the process group's streams their own queues
set -o pipefail
OUT=${1:-gpurun_out/r05rccl2}
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
run q_default "" && run q25 "--hw-queues 25" && run q29 "--hw-queues 29" && run q32 "--hw-queues 32" || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 $X > $OUT/plain.json 2> $OUT/plain.err || { echo "plain failed"; exit 1; }
python -c "
import json
d = json.load(open('$OUT/plain.json')); print('plain', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
