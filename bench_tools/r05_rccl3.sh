#!/bin/bash
# round 5: kernel trace of the RCCL N = 1 bench (one rank, env:// rendezvous, no launcher) beside the
# plain run: which queues the slots' kernels land on, and whether the batches still overlap
set -o pipefail
OUT=${1:-gpurun_out/r05rccl3}
mkdir -p $OUT
export TMPDIR=/tmp
X="--steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29519 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_rccl -o run -- python3 -u bench.py --gpus 1 $X --force-dist > $OUT/rccl.log 2>&1 || { echo "rccl prof failed"; tail -20 $OUT/rccl.log; exit 1; }
unset MASTER_ADDR MASTER_PORT RANK WORLD_SIZE LOCAL_RANK
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_plain -o run -- python3 -u bench.py --gpus 1 $X > $OUT/plain.log 2>&1 || { echo "plain prof failed"; tail -20 $OUT/plain.log; exit 1; }
grep -h -o '"value": [0-9.]*' $OUT/rccl.log $OUT/plain.log
