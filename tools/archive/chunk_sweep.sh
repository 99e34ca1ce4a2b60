#!/bin/bash
# score-kernel chunk sweep for the two-view estimators (solo score ms per batch)
mkdir -p gpurun_out
for est in fundamental essential; do
  for c in ${CHUNK_LIST:-4 8 16 32 64}; do
    timeout -k 10 120 python bench.py --estimator $est --steps 5 --warmup 2 --cpu-seconds 0 --chunks $c > gpurun_out/sweep_${est}_$c.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_${est}_$c.log').read().strip().splitlines()[-1]); print('$est', $c, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],3))"
  done
done
