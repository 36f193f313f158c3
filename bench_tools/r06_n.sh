#!/bin/bash
# round 6: device-side stage stamps of one C2 batch's tail (trace build of the current source)
set -o pipefail
OUT=${1:-gpurun_out/r06n}
mkdir -p $OUT
export TMPDIR=/tmp
SSB_LIB_VARIANT=trace timeout -k 10 150 python -u bench_tools/trace_tail.py > $OUT/trace_tail.txt 2>&1 || { echo "trace tail failed"; grep -v "^W" $OUT/trace_tail.txt | tail -6; exit 1; }
grep -v "^W\|amdgpu.ids" $OUT/trace_tail.txt | grep -v "mf_miller\|mf_group\|TRACE w2" | tail -20
