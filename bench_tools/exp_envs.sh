#!/bin/bash
# Bench at the driver's step count under several settings (one GPU call):
#   bench_tools/exp_envs.sh TAG "VAR=a VAR2=b" "VAR=c#--pipeline 12" ...
# each argument is one run: environment assignments, optionally '#' and extra bench.py flags.
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
k=0
for cfg in "$@"; do
  k=$((k+1))
  envs=${cfg%%#*}; flags=""
  [[ "$cfg" == *"#"* ]] && flags=${cfg#*#}
  env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $flags > $OUT/run$k.json 2> $OUT/run$k.err || { tail -5 $OUT/run$k.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/run$k.json'));print('$cfg |', d['value'], d['ms_per_step'], d['batch_latency_ms'], d['results_ok'], {k: v for k, v in d['kernel_ms'].items() if k.startswith('k_msm') or k in ('k_miller', 'k_final', 'k_hash_to_g2')})"
done
