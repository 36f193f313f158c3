#!/bin/bash
# round 6 (closing): one cursor atomic per distinct digit in the merged G1 sort entries --
# C2 / parity GPU tests, the driver-shaped bench twice, FETCH / WRITE counters of the same bench
set -o pipefail
OUT=${1:-gpurun_out/r06dg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fallback.py -x -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $X --steps 20 > $OUT/b_$rep.json 2> $OUT/b_$rep.err || { echo "bench failed"; tail -5 $OUT/b_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$rep.json')); r=d['roofline']; print('b', $rep, d['value'], d['ms_per_step'], 'sus', d['value_sustained'], 'lat', d['batch_latency_ms'], 'sg_ms', r['avg_launch_ms'], 'frac', r['frac'], 'dec_ms', r['k_decode_count']['avg_launch_ms'], d['results_ok'])"
done
CMD="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --no-adversarial"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pass$i -o run -- $CMD > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pass$i.log; exit 1; }
done
python3 bench_tools/pmc_summary.py $OUT --by-grid > $OUT/summary.json && python3 -c "
import json; d=json.load(open('$OUT/summary.json'))
for k, v in sorted(d.items()):
    if any(x in k for x in ('subgroup_map', 'decode_count<true>@3932', 'msm_bucket2@', 'miller_final')):
        print(k, {c: round(x, 1) for c, x in v.items() if c in ('hbm_bytes_per_launch', 'FETCH_SIZE', 'WRITE_SIZE', 'valu_insts_per_wave', 'SQ_WAVES')})"
