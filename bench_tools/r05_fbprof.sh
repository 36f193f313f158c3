#!/bin/bash
# round 5: kernel traces of the failed-batch patterns at the driver's 20 steps (1e-2 invalid; a faulty
# operator in every committee) beside all-valid
set -o pipefail
OUT=${1:-gpurun_out/r05fbprof}
mkdir -p $OUT
export TMPDIR=/tmp
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --steps 20"
for v in "pct:--invalid-rate 0.01" "badop:--bad-operator 1" "seq:"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$name -o run -- python3 -u bench.py $X $a > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.log; exit 1; }
done
echo done
