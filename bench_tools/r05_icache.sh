#!/bin/bash
# round 5: instruction-fetch counters of the per-share launches (is the subgroup check's ~150 KB loop
# body waiting on the instruction cache?) -- one counter group per rocprofv3 run
set -o pipefail
TAG=${1:-r05ic}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pass$i -o run -- $CMD > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pass$i.log; exit 1; }
done
python3 bench_tools/pmc_summary.py $OUT --by-grid > $OUT/summary.json && python3 -c "
import json; d=json.load(open('$OUT/summary.json'))
for k, v in sorted(d.items()):
    if any(x in k for x in ('subgroup_map@262400', 'decode_count<true>@393216', 'msm_bucket2', 'miller_final')):
        print(k, {c: round(x, 1) for c, x in v.items()})"
