#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, never combined with tracing) over the driver's
# bench command -- the roofline phase's 8 x C2 batch and the pipelined C2 batches are told apart
# by their grid sizes (pmc_summary.py --by-grid).
#   bench_tools/r03_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  GPU_MAX_HW_QUEUES=23 timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pass$i -o run -- $CMD > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pass$i.log; exit 1; }
done
python3 bench_tools/pmc_summary.py $OUT --by-grid > $OUT/summary.json && python3 -c "
import json; d=json.load(open('$OUT/summary.json'))
for k, v in sorted(d.items()):
    if any(x in k for x in ('subgroup_map', 'decode_count', 'bucket2', 'window2', 'miller_final')):
        print(k, {c: round(v.get(c, 0), 3) for c in ('hbm_bytes_per_launch', 'valu_insts_per_wave', 'valu_active_per_busy_cycle', 'SQ_WAVES')})"
rm -rf $OUT/pass1 $OUT/pass2 $OUT/pass3
