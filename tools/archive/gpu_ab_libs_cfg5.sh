#!/bin/bash
# Same-box A/B of cfg5 runs over several library builds: the LO GPU tests through each variant,
# then cfg5 wall time per run (tools/cfg5_split.py, 20 runs) with the builds interleaved.
# usage (gpurun): bash tools/gpu_ab_libs_cfg5.sh <tag> <variant.so>...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for lib in "$@"; do
  RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
      -k "lo or napsac or nonmin or lsq or polish or graphcut" tests > $O/tests.log 2>&1; rc=$?
  echo "$lib tests: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
  for lib in ransac_amd/libransac_amd.so "$@"; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/cfg5_split.py 20 > $O/split.txt 2>&1 || { tail -3 $O/split.txt; exit 1; }
    echo "$lib: $(tail -1 $O/split.txt)"
  done
done
