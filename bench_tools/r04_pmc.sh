#!/bin/bash
# round 4: HBM traffic of the per-share launches, attributed.  FETCH_SIZE and WRITE_SIZE passes (one
# counter per rocprofv3 run, never combined with tracing) over a short bench run -- its roofline batch
# (8 x C2, fused launches) and the C2 batches -- for the product library ("base": the fused launches'
# roles inlined) and the out-of-line-roles build ("outl", SSB_VARIANT=outl SSB_VARIANT_DEFS=-DSSB_ROLES_OUTLINE),
# and once on three-stream slots, where the subgroup checks, the sort's scatter and its count are
# launches of their own (k_subgroup, k_msm_sort, k_decode_sig).
#   bench_tools/r04_pmc.sh TAG
set -o pipefail
TAG=${1:-r04pmc}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
X="--steps 3 --warmup 1 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
run() {   # name, variant, extra bench args
  local name=$1 var=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[pmc] $name $c"
    SSB_LIB_VARIANT=$var timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/$name/$c -o run -- python3 -u bench.py $X "$@" > $OUT/$name.$c.log 2>&1 || { echo "$name $c failed"; tail -20 $OUT/$name.$c.log; exit 1; }
  done
  python3 bench_tools/pmc_summary.py $OUT/$name --by-grid > $OUT/$name.summary.json || exit 1
  rm -rf $OUT/$name
}
run base "" || exit 1
run outl outl || exit 1
run split "" --pipeline 1 --slot-streams 3 || exit 1
python3 - <<EOF
import json
for name in ("base", "outl", "split"):
    d = json.load(open("$OUT/%s.summary.json" % name))
    for k, v in sorted(d.items()):
        if any(x in k for x in ("subgroup", "decode", "msm_sort", "bucket2")):
            print(name, k[:70], "fetch_kb %.0f write_kb %.0f hbm_MB %.1f" % (v.get("FETCH_SIZE", 0), v.get("WRITE_SIZE", 0), v.get("hbm_bytes_per_launch", 0) / 1e6))
EOF
