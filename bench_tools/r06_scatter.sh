#!/bin/bash
# round 6 (closing): XCD-owned scatter of the fused sort (default) against the former per-block form
# (SSB_SCATTER_XCD=0): C2 parity tests, the driver's 20-step command without the side legs
# alternating, then FETCH / WRITE counters of the roofline-shaped bench for both
set -o pipefail
OUT=${1:-gpurun_out/r06sc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial"
for rep in 1 2; do
  for v in owned old; do
    if [ $v = old ]; then export SSB_SCATTER_XCD=0; else unset SSB_SCATTER_XCD; fi
    timeout -k 10 300 python -u bench.py $X --steps 20 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "bench $v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); r=d['roofline']; print('$v', $rep, d['value'], d['ms_per_step'], 'sus', d['value_sustained'], 'lat', d['batch_latency_ms'], 'sg_ms', r['avg_launch_ms'], 'frac', r['frac'], d['results_ok'])"
  done
done
CMD="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --no-adversarial"
for v in owned old; do
  if [ $v = old ]; then export SSB_SCATTER_XCD=0; else unset SSB_SCATTER_XCD; fi
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    echo "[pmc] $v pass $i: $grp"
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/$v/pass$i -o run -- $CMD > $OUT/$v/pass$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/$v/pass$i.log; exit 1; }
  done
  python3 bench_tools/pmc_summary.py $OUT/$v --by-grid > $OUT/$v/summary.json && python3 -c "
import json; d=json.load(open('$OUT/$v/summary.json'))
for k, v in sorted(d.items()):
    if any(x in k for x in ('subgroup_map', 'decode_count', 'msm_bucket2')):
        print('$v', k, {c: round(x, 1) for c, x in v.items() if c in ('hbm_bytes_per_launch', 'FETCH_SIZE', 'WRITE_SIZE')})"
done
unset SSB_SCATTER_XCD
