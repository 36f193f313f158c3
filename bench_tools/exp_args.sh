#!/bin/bash
# Bench under several argument sets (one GPU call):  bench_tools/exp_args.sh TAG "--pipeline 16" "--pipeline 8" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline $a > $OUT/a$i.json 2> $OUT/a$i.err || { tail -20 $OUT/a$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/a$i.json'));print('$a', d['value'], d['ms_per_step'], d['results_ok'], d['value_compressed_pk'])"
done
