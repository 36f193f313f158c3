set -o pipefail
mkdir -p gpurun_out/exp15
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/exp15/tests.log 2>&1 || { tail -40 gpurun_out/exp15/tests.log; exit 1; }
tail -4 gpurun_out/exp15/tests.log
timeout -k 10 300 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline > gpurun_out/exp15/b.json 2> gpurun_out/exp15/b.err || exit 1
