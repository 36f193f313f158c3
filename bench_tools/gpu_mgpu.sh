#!/bin/bash
# One GPU call: the headline bench (driver's arguments), the strong-scaling mode at N=1, and the
# N=2 rehearsal of both modes on ONE GPU over gloo (ranks share the device).
#   bench_tools/gpu_mgpu.sh TAG
set -o pipefail
TAG=${1:-mgpu}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
echo "[mgpu] headline"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/weak1.json 2> $OUT/weak1.err || { tail -20 $OUT/weak1.err; exit 1; }
cut -c1-400 $OUT/weak1.json
echo "[mgpu] strong N=1"
timeout -k 10 400 python -u bench.py --scaling strong --steps 6 --warmup 2 --no-cpu-baseline > $OUT/strong1.json 2> $OUT/strong1.err || { tail -20 $OUT/strong1.err; exit 1; }
cut -c1-400 $OUT/strong1.json
for MODE in weak strong; do
  echo "[mgpu] gloo N=2 $MODE"
  timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --steps 6 --warmup 2 --scaling $MODE --dist-backend gloo --pipeline 4 > $OUT/gloo2_$MODE.json 2> $OUT/gloo2_$MODE.err || { tail -30 $OUT/gloo2_$MODE.err; exit 1; }
  cut -c1-400 $OUT/gloo2_$MODE.json
done
