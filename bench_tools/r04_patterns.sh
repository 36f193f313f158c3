#!/bin/bash
# the invalid-share patterns and registry ids at the default length (200 timed steps)
set -o pipefail
OUT=${1:-gpurun_out/r04pat}; mkdir -p $OUT
X="--no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "one:--invalid-count 1" "pct1:--invalid-rate 0.01" "badop:--bad-operator 2" "registry:--ids registry" "registry_one:--ids registry --invalid-count 1"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['steps'], d['results_ok'], d['invalid_shares_per_batch'], d['batch_latency_ms'])"
done
