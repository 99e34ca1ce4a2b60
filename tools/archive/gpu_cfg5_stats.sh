#!/bin/bash
# cfg5 per-seed statistics for the current build and variants: bash tools/gpu_cfg5_stats.sh <variant.so>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ransac_amd/libransac_amd.so "$@"; do
  RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 200 python tools/cfg5_stats.py 100 > gpurun_out/c5s.txt 2>&1 || { tail -3 gpurun_out/c5s.txt; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/c5s.txt)"
done
