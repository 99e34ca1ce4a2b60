#!/bin/bash
# same-box A/B of the HIP hardware-queue count (GPU_MAX_HW_QUEUES 4 = default vs Q) on a bench line
# usage (gpurun): bash tools/gpu_q_ab.sh <tag> <Q> [bench args...]
set -o pipefail
TAG=$1; Q=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2 3; do
  for q in 4 $Q; do
    timeout -k 10 180 env GPU_MAX_HW_QUEUES=$q python bench.py --steps 100 --warmup 10 --cpu-seconds 0 "$@" > $O/q.log 2> $O/q.err || { tail -3 $O/q.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/q.log').read().strip().splitlines()[-1]); print('queues %2d %-40s %8.2f M/s ms/step %.4f parity %s' % ($q, '$*', d['value']/1e6, d['ms_per_step'], d['parity'].get('scores_bit_equal', d['parity'].get('model_bit_equal'))))" | tee -a $O/q.txt
  done
done
