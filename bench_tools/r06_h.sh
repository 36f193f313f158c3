#!/bin/bash
# round 6: kernel-trace summaries (rocprofv3 --kernel-trace --stats) of the driver command and of the
# faulty-operator / 1e-2 patterns, then HBM and SQ counters (one group per pass, never with tracing)
# over the roofline-shaped bench (pmc_summary.py --by-grid tells the roofline batch from the C2 ones)
set -o pipefail
OUT=${1:-gpurun_out/r06h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/drv -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv.json 2> $OUT/drv.err || { echo "driver prof failed"; tail -5 $OUT/drv.err; exit 1; }
X="--warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --no-adversarial --steps 20"
for v in "badop:--bad-operator 1" "pct:--invalid-rate 0.01"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run -- python3 -u bench.py $X $a > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
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
    if any(x in k for x in ('subgroup_map', 'decode_count', 'miller_final', 'msm_bucket2')):
        print(k, {c: round(x, 1) for c, x in v.items() if c in ('hbm_bytes_per_launch', 'valu_insts_per_wave', 'SQ_WAVES')})"
