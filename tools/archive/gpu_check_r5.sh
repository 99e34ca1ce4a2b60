#!/bin/bash
# Round-5 check on one GPU: every -m gpu test, then the N = 2 rehearsal of bench.py's multi-rank
# lines (tools/gpu_multi_rehearsal.sh).  Usage (GPU box): bash tools/gpu_check_r5.sh <tag>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_multi_rehearsal.sh ${1:-r5}/multi
