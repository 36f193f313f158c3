#!/bin/bash
# round 5: the failed-batch chain's kernels for ONE batch alone (pipeline depth 1): which launches
# make the one-invalid / 1e-2 / faulty-operator latency
set -o pipefail
OUT=${1:-gpurun_out/r05fblat}
mkdir -p $OUT
export TMPDIR=/tmp
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --steps 6 --pipeline 1"
for v in "one:--invalid-count 1" "pct:--invalid-rate 0.01" "badop:--bad-operator 1"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$name -o run -- python3 -u bench.py $X $a > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.log; exit 1; }
done
echo done
