#!/bin/bash
# round 5: the headline path, round-4 HEAD (ab_r4/, built from 5620e00) against this tree on one box,
# interleaved, then a kernel-trace profile of each (which kernels got slower)
set -o pipefail
OUT=${1:-gpurun_out/r05ab}
mkdir -p $OUT
export TMPDIR=/tmp
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --steps 20"
for i in 1 2; do
  (cd ab_r4 && timeout -k 10 300 python -u bench.py $X > ../$OUT/r4_$i.json 2> ../$OUT/r4_$i.err) || { echo "r4 bench failed"; tail -5 $OUT/r4_$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py $X --no-registry > $OUT/r5_$i.json 2> $OUT/r5_$i.err || { echo "r5 bench failed"; tail -5 $OUT/r5_$i.err; exit 1; }
  python -c "
import json
for n in ('r4_$i', 'r5_$i'):
    d = json.load(open('$OUT/%s.json' % n)); print(n, d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
done
(cd ab_r4 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../$OUT/prof_r4 -o run -- python3 -u bench.py $X > ../$OUT/prof_r4.log 2>&1) || { echo "r4 prof failed"; tail -5 $OUT/prof_r4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r5 -o run -- python3 -u bench.py $X --no-registry > $OUT/prof_r5.log 2>&1 || { echo "r5 prof failed"; tail -5 $OUT/prof_r5.log; exit 1; }
echo done
