set -o pipefail
mkdir -p gpurun_out/exp8
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/exp8/tests.log 2>&1 || { tail -30 gpurun_out/exp8/tests.log; exit 1; }
tail -1 gpurun_out/exp8/tests.log
B="python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline"
for cfg in "16 1" "12 1" "24 1" "8 3"; do
  set -- $cfg
  timeout -k 10 200 $B --pipeline $1 --slot-streams $2 > gpurun_out/exp8/p$1s$2.json 2> gpurun_out/exp8/p$1s$2.err
  rc=$?; echo "pipeline $1 streams $2 rc=$rc"; grep -h "OUT_OF_RES" gpurun_out/exp8/p$1s$2.err | head -1 | cut -c1-120
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
