#!/bin/bash
# A/B a variant library on all three bench estimators (solo kernel ms)
V=$1
for est in homography fundamental essential; do
  for lib in ransac_amd/libransac_amd.so $V; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --estimator $est --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s %-36s %8.2f M/s score %.4f solve %.4f parity %s' % ('$est', '$lib', d['value']/1e6, r['kernel_ms'], r['solve_kernel_ms'], d['parity']['scores_bit_equal']))"
  done
done
