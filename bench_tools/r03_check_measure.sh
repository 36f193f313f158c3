#!/bin/bash
# One GPU call: the -m gpu tests, then bench_tools/r03_measure.sh TAG (stops at the first failure).
set -o pipefail
TAG=$1; shift; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -2 gpurun_out/$TAG/tests.log
bench_tools/r03_measure.sh $TAG "$@"
