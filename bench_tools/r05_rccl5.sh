#!/bin/bash
# round 5: host submit times and per-batch start/end on the slot streams, RCCL N = 1 vs plain
set -o pipefail
OUT=${1:-gpurun_out/r05rccl5}
mkdir -p $OUT
X="--steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
export SSB_DEBUG_HOST=1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 1 $X --force-dist > $OUT/d.json 2> $OUT/d.err || { echo "d failed"; tail -20 $OUT/d.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 $X > $OUT/p.json 2> $OUT/p.err || { echo "p failed"; tail -20 $OUT/p.err; exit 1; }
grep -h "host ms\|batch start" $OUT/d.err | tail -2
grep -h "host ms\|batch start" $OUT/p.err | tail -2
