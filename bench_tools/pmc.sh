#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, never combined with tracing) over a short
# depth-1 bench run; then bench_tools/pmc_summary.py -> profiles/pmc_*.json
#   bench_tools/pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 -u bench.py --steps 2 --warmup 1 --pipeline 1 --slot-streams 3 --no-cpu-baseline --no-host-buffers"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/pass$i -o run -- $CMD > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pass$i.log; exit 1; }
done
find $OUT -name '*counter_collection.csv' | head
python3 bench_tools/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
