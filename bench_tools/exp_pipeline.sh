set -o pipefail
mkdir -p gpurun_out/exp14
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 500 --timeout-method thread -k "large_configs" > gpurun_out/exp14/tests.log 2>&1 || { tail -40 gpurun_out/exp14/tests.log; exit 1; }
tail -4 gpurun_out/exp14/tests.log
