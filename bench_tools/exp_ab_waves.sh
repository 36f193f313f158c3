set -o pipefail
OUT=gpurun_out/r02s4_ab_waves; mkdir -p $OUT
for r in 1 2; do for v in base sg3 b23; do
  if [ "$v" = base ]; then export SSB_LIB_VARIANT=; else export SSB_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { tail -20 $OUT/$v.$r.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$v.$r.json'));print('$v', $r, d['value'], d['ms_per_step'], d['results_ok'])"
done; done
