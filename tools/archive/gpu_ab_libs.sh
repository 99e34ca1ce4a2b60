#!/bin/bash
# Same-box A/B of a bench line over several library builds: the selected GPU tests through each
# build, then bench.py lines with the builds interleaved (3 reps).
# usage (gpurun): bash tools/gpu_ab_libs.sh <tag> <estimator> <pytest -k expr> <variant.so>...
set -o pipefail
TAG=$1; EST=$2; K=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for lib in ransac_amd/libransac_amd.so "$@"; do
  RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
      -k "$K" tests > $O/tests.log 2>&1; rc=$?
  echo "$lib tests: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
  for lib in ransac_amd/libransac_amd.so "$@"; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 180 python bench.py --estimator $EST --steps 100 --warmup 10 --cpu-seconds 0 > $O/ab.log 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%-34s %8.2f M/s ms/step %.4f score %.4f solve %.4f parity %s' % ('$lib', d['value']/1e6, d['ms_per_step'], r.get('kernel_ms'), r.get('solve_kernel_ms'), d['parity'].get('scores_bit_equal')))" | tee -a $O/ab.txt
  done
done
