#!/bin/bash
# round 6: the GPU suite on the library with the restructured fallback / combine frames, then the
# profiling call (r06_h.sh: kernel traces of the driver command and the failed-batch patterns, PMC)
set -o pipefail
OUT=${1:-gpurun_out/r06i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash bench_tools/r06_h.sh $OUT
