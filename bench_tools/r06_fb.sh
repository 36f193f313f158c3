#!/bin/bash
# round 6: the 28-bit product microbenchmark, then the group-test item counter of k_fb_excl: the GPU
# fallback tests on the product library, the faulty-operator batch through the trace build with
# bounds checks (SSB_FB_CHECKS), and the driver-shaped faulty-operator bench
set -o pipefail
OUT=${1:-gpurun_out/r06fb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./bench_tools/r28_bench > $OUT/r28.json 2> $OUT/r28.err || { echo "r28 failed"; tail -5 $OUT/r28.err; exit 1; }
python3 bench_tools/r28_check.py < $OUT/r28.json || echo "r28 samples WRONG"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fallback.py -x -v --timeout 150 --timeout-method thread > $OUT/fb_tests.log 2>&1 || { echo "fallback tests failed"; tail -30 $OUT/fb_tests.log; exit 1; }
tail -1 $OUT/fb_tests.log
for i in 1 2; do
  SSB_LIB_VARIANT=trace timeout -k 10 150 python -u bench_tools/trace_fb.py badop > $OUT/trace_badop$i.txt 2>&1 || { echo "trace badop $i failed"; grep -v "^W" $OUT/trace_badop$i.txt | tail -6; exit 1; }
  grep -v "^W\|amdgpu.ids" $OUT/trace_badop$i.txt
done
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --no-adversarial"
timeout -k 10 300 python -u bench.py $X --steps 20 --bad-operator 1 > $OUT/badop20.json 2> $OUT/badop20.err || { echo "bench badop failed"; tail -5 $OUT/badop20.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/badop20.json')); print('badop20', d['value'], d['ms_per_step'], d['results_ok'])"
