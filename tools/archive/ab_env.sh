#!/bin/bash
# A/B of an environment switch on the default bench (same box, interleaved): prints hyp/s and
# the score / solve kernels' solo ms.   usage: ab_env.sh VAR [bench args...]
VAR=$1; shift
mkdir -p gpurun_out
for rep in 1 2 3; do
  for val in 0 1; do
    env $VAR=$val timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 "$@" > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%s=%s %8.2f M/s score %.4f solve %.4f parity %s' % ('$VAR', '$val', d['value']/1e6, r['kernel_ms'], r['solve_kernel_ms'], d['parity']))"
  done
done
