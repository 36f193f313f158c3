#!/bin/bash
# Single-lane vs 8-lane-group subgroup checks (SSB_SUBGROUP): GPU tests, then the C2 bench at depths.
#   bench_tools/exp_subgroup.sh TAG "14 16"
set -o pipefail
TAG=${1:-subgroup}; DEPTHS=${2:-"14"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "subgroup or golden" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for sg in single lane; do
  for d in $DEPTHS; do
    SSB_SUBGROUP=$sg timeout -k 10 240 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline --pipeline $d > $OUT/$sg-d$d.json 2> $OUT/$sg-d$d.err || { tail -20 $OUT/$sg-d$d.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$sg-d$d.json'));print('$sg', $d, d['value'], d['ms_per_step'], d['batch_latency_ms'], d['kernel_ms']['k_subgroup'], d['roofline']['frac'])"
  done
done
