#!/bin/bash
# round 6: device-side stage stamps of one C2 batch's tail (trace build of the current source,
# SSB_VARIANT_DEFS=-DSSB_TRACE_TAIL), then the faulty-operator batch through the same build
set -o pipefail
OUT=${1:-gpurun_out/r06l}
mkdir -p $OUT
export TMPDIR=/tmp
SSB_LIB_VARIANT=trace timeout -k 10 150 python -u bench_tools/trace_tail.py > $OUT/trace_tail.txt 2>&1 || { echo "trace tail failed"; grep -v "^W" $OUT/trace_tail.txt | tail -6; exit 1; }
grep -v "^W\|amdgpu.ids" $OUT/trace_tail.txt | tail -40
SSB_LIB_VARIANT=trace timeout -k 10 150 python -u bench_tools/trace_fb.py badop > $OUT/trace_badop.txt 2>&1 || { echo "trace badop failed"; grep -v "^W" $OUT/trace_badop.txt | tail -6; exit 1; }
grep -v "^W\|amdgpu.ids" $OUT/trace_badop.txt | tail -20
