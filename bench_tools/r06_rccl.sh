#!/bin/bash
# round 6: RCCL at N = 1 (process group 'nccl', the exchange issued by bench.py's Exchanger thread on
# finished batches) against the plain run, alternating, the 20-step value and 1,000 sustained steps
set -o pipefail
OUT=${1:-gpurun_out/r06rccl}
mkdir -p $OUT
X="--steps 20 --warmup 5 --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 1000 --no-registry --no-adversarial"
for rep in 1 2; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
      bench.py --gpus 1 $X --force-dist > $OUT/d$rep.json 2> $OUT/d$rep.err || { echo "rccl $rep failed"; tail -20 $OUT/d$rep.err; exit 1; }
  timeout -k 10 300 python -u bench.py --gpus 1 $X > $OUT/p$rep.json 2> $OUT/p$rep.err || { echo "plain $rep failed"; tail -20 $OUT/p$rep.err; exit 1; }
  for k in d p; do
    python3 -c "
import json
d = json.loads(open('$OUT/$k$rep.json').read().strip().splitlines()[-1])
print('$k', $rep, d['value'], d['ms_per_step'], 'sus', d.get('value_sustained'), 'lat', d.get('batch_latency_ms'), d.get('config', {}).get('parallelism'), d['results_ok'])"
  done
done
