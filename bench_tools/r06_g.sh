#!/bin/bash
# round 6: the GPU suite, smoke and the driver bench (r06_check.sh), then RCCL at N = 1 against the
# plain run (r06_rccl.sh)
set -o pipefail
OUT=${1:-gpurun_out/r06g}
bash bench_tools/r06_check.sh $OUT && bash bench_tools/r06_rccl.sh $OUT
