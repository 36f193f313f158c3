#!/bin/bash
# round 4: the BASELINE.json configs beyond the headline (one bench line each), then the multi-rank
# rehearsal on one GPU: bench.py --gpus 2 over gloo (it launches its two ranks itself)
set -o pipefail
OUT=${1:-gpurun_out/r04cfg}; mkdir -p $OUT
for c in C3_3of4 C3_5of7 C4_per_gpu C5_per_gpu; do
  timeout -k 10 400 python -u bench.py --config $c --steps 6 --warmup 1 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 > $OUT/$c.json 2> $OUT/$c.err || { tail -20 $OUT/$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', d['value'], d['combined_sigs_per_s'], d['ms_per_step'], d['results_ok'], d['batch_latency_ms'], d['step_roofline']['frac'])"
done
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -20 $OUT/gloo2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/gloo2.json'));print('gloo2', d['n_gpus'], d['value'], d['ms_per_step'], d['results_ok'], d['config'])"
