#!/bin/bash
# Round 6: latency forms of the MSM launches at depth 1 (lane-program G2 window sums, clearing beside
# the bucket sums): parity vs the C oracle, then the driver's command with and without them.
mkdir -p gpurun_out/r06u
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py \
  -k "depth1_latency or (cached_one_stream_matches and merged)" > gpurun_out/r06u/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r06u/tests.log; exit 1; }
tail -3 gpurun_out/r06u/tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06u/bench_lat.json 2> gpurun_out/r06u/bench_lat.err || { echo "bench rc=$?"; tail -20 gpurun_out/r06u/bench_lat.err; exit 1; }
SSB_MSM_LAT=0 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06u/bench_nolat.json 2> gpurun_out/r06u/bench_nolat.err || { echo "bench2 rc=$?"; exit 1; }
python3 - <<'PY'
import json
for f in ["bench_lat", "bench_nolat"]:
    d = json.loads(open("gpurun_out/r06u/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["batch_latency_ms"], d["batch_latency_ms_by_config"], d["kernel_ms"]["k_msm_g2"], d.get("value_sustained"))
PY
