#!/bin/bash
# batches-in-flight sweep per estimator (same box, interleaved reps): bench.py --pipeline P
# usage (gpurun): bash tools/gpu_pipe_sweep.sh <tag> "<estimators>" "<depths>"
set -o pipefail
TAG=$1; ESTS=${2:-"fundamental essential homography"}; DEPTHS=${3:-"2 3 4 6 8"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for est in $ESTS; do
  for rep in 1 2; do
    for p in $DEPTHS; do
      timeout -k 10 180 env ${QENV:-} python bench.py --estimator $est --pipeline $p --steps 100 --warmup 10 --cpu-seconds 0 > $O/sw.log 2> $O/sw.err || { tail -3 $O/sw.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/sw.log').read().strip().splitlines()[-1]); print('%-12s pipeline %d  %8.2f M/s ms/step %.4f parity %s' % ('$est', $p, d['value']/1e6, d['ms_per_step'], d['parity'].get('scores_bit_equal')))" | tee -a $O/sweep.txt
    done
  done
done
