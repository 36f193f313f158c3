#!/bin/bash
# round 5, late: the final validation (GPU suite, smoke, driver bench + rocprof stats) and the fallback
# patterns on the final library, then the fallback traces (experiment build) last
set -o pipefail
OUT=${1:-gpurun_out/r05final2}
bash bench_tools/r05_final.sh $OUT || exit 1
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
for v in "pct20:--steps 20 --invalid-rate 0.01" "one20:--steps 20 --invalid-count 1" "badop20:--steps 20 --bad-operator 1"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
done
for p in badop pct; do
  SSB_LIB_VARIANT=trace timeout -k 10 150 python -u bench_tools/trace_fb.py $p > $OUT/trace_$p.txt 2>&1 || { echo "trace $p failed"; tail -5 $OUT/trace_$p.txt; exit 1; }
  grep -v "^W\|amdgpu.ids" $OUT/trace_$p.txt
done
