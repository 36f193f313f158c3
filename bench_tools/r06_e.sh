#!/bin/bash
# round 6: the faulty-operator batch three times on one slot (bench_tools/trace_fb.py's scenario) through
# the PRODUCT library, then the driver-shaped faulty-operator bench, the reduced-radix A/B (r06_ab.sh)
# and the GPU suite / smoke / driver bench (r06_check.sh)
set -o pipefail
OUT=${1:-gpurun_out/r06e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python -u bench_tools/trace_fb.py badop > $OUT/product_badop.txt 2>&1 || { echo "product badop failed"; grep -v "^W" $OUT/product_badop.txt | tail -6; exit 1; }
grep -v "^W\|amdgpu.ids" $OUT/product_badop.txt
X="--warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0 --no-registry --no-adversarial"
timeout -k 10 300 python -u bench.py $X --steps 20 --bad-operator 1 > $OUT/badop20.json 2> $OUT/badop20.err || { echo "bench badop failed"; tail -5 $OUT/badop20.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/badop20.json')); print('badop20', d['value'], d['ms_per_step'], d['results_ok'])"
bash bench_tools/r06_ab.sh $OUT && bash bench_tools/r06_check.sh $OUT
