#!/bin/bash
# kernel durations of 1e-2 batches run one at a time (depth 1): the fallback chain on an idle chip
set -o pipefail
OUT=${1:-gpurun_out/r04lat}; mkdir -p $OUT
PROF_X="--steps 4 --warmup 1" bash bench_tools/r04_prof.sh $OUT "pct1d1:--invalid-rate 0.01 --pipeline 1"
