set -o pipefail
mkdir -p gpurun_out/exp3
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/exp3/prof -o run -- python3 -u bench.py --steps 12 --warmup 4 --no-cpu-baseline --pipeline 4 > gpurun_out/exp3/p4.json 2> gpurun_out/exp3/p4.err || exit 1
