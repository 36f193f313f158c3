#!/bin/bash
# Bench under (environment, arguments) pairs, one GPU call:
#   bench_tools/exp_mix.sh TAG "ENV=a,ENV2=b|--pipeline 14" "-|--pipeline 12" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for spec in "$@"; do
  i=$((i+1))
  setting=${spec%%|*}; args=${spec#*|}
  envs=(); [ "$setting" != "-" ] && IFS=',' read -ra envs <<< "$setting"
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline $args > $OUT/m$i.json 2> $OUT/m$i.err || { tail -20 $OUT/m$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/m$i.json'));print('$spec', d['value'], d['ms_per_step'], d['results_ok'], d['value_compressed_pk'])"
done
