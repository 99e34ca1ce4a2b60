#!/bin/bash
# cfg4 score-kernel A/B: base library over chunk counts, then the variant builds (var_libs/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
O=gpurun_out/ab_score_e.jsonl; : > $O
CHUNKS=48,96,128 timeout -k 10 180 python3 tools/archive/ab_score_e.py >> $O || exit 1
for v in "$@"; do
  RANSAC_AMD_LIB=$PWD/ransac_amd/var_libs/lib_$v.so CHUNKS=96 timeout -k 10 180 python3 tools/archive/ab_score_e.py >> $O || exit 1
done
cat $O
