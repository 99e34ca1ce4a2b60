#!/bin/bash
# NAPSAC grid build + download wall time and the cfg5 setup split, current library vs a variant
#   bash tools/gpu_grid_time.sh <variant.so>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for lib in ransac_amd/libransac_amd.so $1; do
    echo "$lib: $(RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/grid_time.py 20)"
    USAC_PROFILE=1 RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/cfg5_split.py 20 2>&1 | grep "usac_ransac_run" | tail -1
  done
done
