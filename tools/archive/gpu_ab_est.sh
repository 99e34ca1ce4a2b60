#!/bin/bash
# Same-box A/B of library variants on one estimator's bench line: bash tools/gpu_ab_est.sh <tag> <estimator> <variant.so>...
set -o pipefail
TAG=$1; EST=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for lib in ransac_amd/libransac_amd.so "$@"; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 180 python bench.py --estimator $EST --steps 100 --warmup 10 --cpu-seconds 0 > $O/ab.log 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab.log').read().strip().splitlines()[-1]); print('%-34s %8.2f M/s ms/step %.4f parity %s' % ('$lib', d['value']/1e6, d['ms_per_step'], d['parity'].get('timed_kernel',{}).get('ok')))"
  done
done
