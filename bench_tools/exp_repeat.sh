#!/bin/bash
# Reliability / spread of the driver's bench command: K runs of bench.py --steps 20 --warmup 5
# (no CPU baseline), stop at the first failure.
#   bench_tools/exp_repeat.sh TAG K ["ENV=val ..."]
set -o pipefail
TAG=$1; K=${2:-10}; ENVS=${3:-SSB_X=0}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $K); do
  env $ENVS timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers > $OUT/run$i.json 2> $OUT/run$i.err || { echo "run $i FAILED"; grep -m3 -i "error" $OUT/run$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/run$i.json'));print('run $i', d['value'], d['ms_per_step'], d['results_ok'])"
done
