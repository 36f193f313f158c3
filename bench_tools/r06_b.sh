#!/bin/bash
# round 6, second call: the 28-bit product microbenchmark and the k_fb_excl item counter first
# (r06_fb.sh), then the GPU suite, smoke and the driver bench (r06_check.sh)
set -o pipefail
OUT=${1:-gpurun_out/r06b}
bash bench_tools/r06_fb.sh $OUT && bash bench_tools/r06_check.sh $OUT
