#!/bin/bash
# cfg2 score-kernel A/B: base library and variant builds (var_libs/), interleaved, 3 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
O=gpurun_out/ab_score_h.jsonl; : > $O
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/archive/ab_score_h.py >> $O || exit 1
  for v in "$@"; do
    RANSAC_AMD_LIB=$PWD/ransac_amd/var_libs/lib_$v.so timeout -k 10 120 python3 tools/archive/ab_score_h.py >> $O || exit 1
  done
done
cat $O
