#!/bin/bash
# Bench under several environment settings (one GPU call):
#   bench_tools/exp_env.sh TAG RATE "ENV1=a,ENV2=b" "ENV1=c" ...
# (each setting: comma-separated VAR=VALUE pairs; "-" = no extra environment)
set -o pipefail
TAG=$1; RATE=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for setting in "$@"; do
  i=$((i+1))
  envs=(); [ "$setting" != "-" ] && IFS=',' read -ra envs <<< "$setting"
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 36 --warmup 2 --no-cpu-baseline --invalid-rate $RATE > $OUT/e$i.json 2> $OUT/e$i.err || { tail -20 $OUT/e$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/e$i.json'));print('$setting rate $RATE', d['value'], d['ms_per_step'], d['results_ok'], d['kernel_ms']['k_fallback_verify'])"
done
