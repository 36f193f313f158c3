#!/bin/bash
# Round 6: fallback grid caps (k_fb_single, k_fb_level) A/B on the driver's command, two alternations.
mkdir -p gpurun_out/r06x
for r in 1 2; do
  for cfg in "512,512" "128,128" "64,64"; do
    SSB_FB_GRID=$cfg timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06x/b_${cfg/,/_}_$r.json 2> gpurun_out/r06x/b_${cfg/,/_}_$r.err || { echo "bench $cfg rc=$?"; tail -5 gpurun_out/r06x/b_${cfg/,/_}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06x/b_${cfg/,/_}_$r.json').read().strip().splitlines()[-1])
print('$cfg', $r, d['value'], d['value_invalid_1e2'], d['value_bad_operator'], d['results_ok'], d['adversarial']['invalid_1e2']['results_ok'], d['adversarial']['bad_operator']['results_ok'])"
  done
done
