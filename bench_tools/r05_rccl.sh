#!/bin/bash
# round 5: the whole GPU suite, then the RCCL path at N = 1 (torchrun, one rank, --force-dist:
# the all-gather of verdicts + signatures on RCCL's stream beside the 20 slot queues) next to the
# non-distributed run of the same command
set -o pipefail
OUT=${1:-gpurun_out/r05rccl}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 $A --force-dist > $OUT/n1_rccl.json 2> $OUT/n1_rccl.err || { echo "rccl n1 failed"; tail -20 $OUT/n1_rccl.err; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 1 $A > $OUT/n1_plain.json 2> $OUT/n1_plain.err || { echo "plain n1 failed"; tail -20 $OUT/n1_plain.err; exit 1; }
python -c "
import json
for n in ('n1_rccl', 'n1_plain'):
    d = json.loads(open('$OUT/%s.json' % n).read().strip().splitlines()[-1])
    print(n, {k: d.get(k) for k in ('value', 'ms_per_step', 'value_registry', 'value_collector', 'value_collector_wire', 'batch_latency_ms', 'results_ok')}, d['config'].get('parallelism'))"
