#!/bin/bash
# Round 6: device stamps of one C2 batch at depth 1 with the MSM latency forms (default) and without
# (SSB_MSM_LAT=0), experiment build with trace stamps.
mkdir -p gpurun_out/r06v
export SSB_LIB_VARIANT=trace
timeout -k 10 300 python -u bench_tools/trace_tail.py > gpurun_out/r06v/trace_lat.txt 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/r06v/trace_lat.txt; exit 1; }
SSB_MSM_LAT=0 timeout -k 10 300 python -u bench_tools/trace_tail.py > gpurun_out/r06v/trace_nolat.txt 2>&1 || { echo "rc=$?"; exit 1; }
python bench_tools/trace_tail.py --summarize gpurun_out/r06v/trace_lat.txt | tail -14
echo ---
python bench_tools/trace_tail.py --summarize gpurun_out/r06v/trace_nolat.txt | tail -14
