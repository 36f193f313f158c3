#!/bin/bash
# round 6, third call: microbenchmark + item counter (r06_fb.sh), the subgroup A/B (r06_ab.sh), then the
# GPU suite, smoke and the driver bench (r06_check.sh)
set -o pipefail
OUT=${1:-gpurun_out/r06c}
bash bench_tools/r06_fb.sh $OUT && bash bench_tools/r06_ab.sh $OUT && bash bench_tools/r06_check.sh $OUT
