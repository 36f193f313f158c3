#!/bin/bash
# registry ids after the cheaper ratio combine: GPU parity (fallback + registry tests), then the driver's
# C2 command for seq / registry ids, then kernel profiles
set -o pipefail
OUT=${1:-gpurun_out/r04reg2}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fallback.py -x -v --timeout 200 --timeout-method thread -m gpu -k "registry or knobs" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--steps 20 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "valid:" "registry:--ids registry"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['results_ok'], {k: round(v, 3) for k, v in d['kernel_ms'].items() if v > 0.05})"
done
bash bench_tools/r04_prof.sh $OUT "registry:--ids registry" "pct1:--invalid-rate 0.01"
