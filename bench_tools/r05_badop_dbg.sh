#!/bin/bash
# round 5: the faulty-operator batch at depth 1 on the product library (verdicts of three batches),
# the badop bench, then the trace build once under a kernel trace (which launch faults)
set -o pipefail
OUT=${1:-gpurun_out/r05dbg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u bench_tools/trace_fb.py badop > $OUT/product_badop.txt 2>&1 || { echo "product badop failed"; tail -8 $OUT/product_badop.txt; exit 1; }
grep -v "^W\|amdgpu.ids" $OUT/product_badop.txt
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
timeout -k 10 300 python -u bench.py $X --steps 20 --bad-operator 1 > $OUT/badop20.json 2> $OUT/badop20.err || { echo "bench badop failed"; tail -5 $OUT/badop20.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/badop20.json')); print('badop20', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'])"
export SSB_LIB_VARIANT=trace
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/trace_kt -o run -- python3 -u bench_tools/trace_fb.py badop > $OUT/trace_badop.txt 2>&1 || { echo "trace badop failed"; grep -v "^W" $OUT/trace_badop.txt | tail -4; exit 1; }
grep -v "^W\|amdgpu.ids" $OUT/trace_badop.txt
