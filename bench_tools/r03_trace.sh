#!/bin/bash
# Tail critical path of one C2 batch (bench_tools/trace_tail.py, experiment build libssbls_trace.so).
set -o pipefail
mkdir -p gpurun_out/r03_tr
SSB_LIB_VARIANT=trace timeout -k 10 200 python -u bench_tools/trace_tail.py > gpurun_out/r03_tr/trace.txt 2> gpurun_out/r03_tr/trace.err && python bench_tools/trace_tail.py --summarize gpurun_out/r03_tr/trace.txt
