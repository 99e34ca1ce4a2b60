#!/bin/bash
# A/B of two library builds on the default bench (score-kernel solo ms + pipelined hyp/s)
# usage: ab_lib.sh <variant.so> [bench args...]
V=$1; shift
mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in ransac_amd/libransac_amd.so ransac_amd/var_libs/lib_$V.so; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 "$@" > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%-40s %8.2f M/s score %.4f solve %.4f parity %s' % ('$lib', d['value']/1e6, r['kernel_ms'], r['solve_kernel_ms'], d['parity']['scores_bit_equal']))"
  done
done
