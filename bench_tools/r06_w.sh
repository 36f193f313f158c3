#!/bin/bash
# Round 6: MSM latency forms after the digit-0 fix: device stamps, parity, driver command A/B.
mkdir -p gpurun_out/r06w
SSB_LIB_VARIANT=trace timeout -k 10 300 python -u bench_tools/trace_tail.py > gpurun_out/r06w/trace_lat.txt 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/r06w/trace_lat.txt; exit 1; }
python bench_tools/trace_tail.py --summarize gpurun_out/r06w/trace_lat.txt | tail -14
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py \
  -k "depth1_latency or (cached_one_stream_matches and merged)" > gpurun_out/r06w/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r06w/tests.log; exit 1; }
tail -2 gpurun_out/r06w/tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06w/bench_lat.json 2> gpurun_out/r06w/bench_lat.err || { echo "bench rc=$?"; tail -20 gpurun_out/r06w/bench_lat.err; exit 1; }
SSB_MSM_LAT=0 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06w/bench_nolat.json 2> gpurun_out/r06w/bench_nolat.err || { echo "bench2 rc=$?"; exit 1; }
python3 - <<'PY'
import json
for f in ["bench_lat", "bench_nolat"]:
    d = json.loads(open("gpurun_out/r06w/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["batch_latency_ms"], d["batch_latency_ms_by_config"], d.get("value_sustained"), d.get("value_invalid_1e2"), d.get("value_bad_operator"))
PY
