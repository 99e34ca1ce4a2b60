#!/bin/bash
# GPU tests + solve-stage A/B of the current library against a variant build.
# usage (gpurun): bash tools/gpu_ab_solve.sh <tag> <variant.so> [pytest -k expr]
set -o pipefail
TAG=$1; V=$2; K=${3:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
fi
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for est in homography fundamental essential; do
  for rep in 1 2; do
    for lib in ransac_amd/libransac_amd.so $V; do
      RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 180 python bench.py --estimator $est --steps 50 --warmup 5 --cpu-seconds 0 > $O/ab.log 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s %-34s %8.2f M/s ms/step %.4f score %s solve %s parity %s' % ('$est', '$lib', d['value']/1e6, d['ms_per_step'], r.get('kernel_ms'), r.get('solve_kernel_ms'), d['parity'].get('scores_bit_equal')))"
    done
  done
done
