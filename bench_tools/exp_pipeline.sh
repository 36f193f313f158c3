set -o pipefail
mkdir -p gpurun_out/exp13
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/exp13/tests.log 2>&1 || { tail -30 gpurun_out/exp13/tests.log; exit 1; }
tail -1 gpurun_out/exp13/tests.log
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=20
timeout -k 10 200 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline > gpurun_out/exp13/plain.json 2> gpurun_out/exp13/plain.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp13/prof -o run -- python3 -u bench.py --steps 48 --warmup 2 --no-cpu-baseline > gpurun_out/exp13/b.json 2> gpurun_out/exp13/b.err || exit 1
