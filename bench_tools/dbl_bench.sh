set -o pipefail
mkdir -p gpurun_out/dbl
for v in 0 3; do
  timeout -k 10 120 ./bench_tools/dbl_bench_v$v > gpurun_out/dbl/v$v.json || exit 1
  echo "v$v $(cat gpurun_out/dbl/v$v.json)"
done
