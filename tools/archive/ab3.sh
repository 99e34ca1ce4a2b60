#!/bin/bash
# score-kernel timing of library variants (no parity meaning for experiment builds)
for lib in "$@"; do
  RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --estimator essential --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%-44s %8.2f M/s score %.4f solve %.4f' % ('$lib', d['value']/1e6, r['kernel_ms'], r['solve_kernel_ms']))"
done
