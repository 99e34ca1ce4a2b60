#!/bin/bash
# Grid-build check: the grid / NAPSAC GPU tests, then a same-box A/B of cfg5 runs between the
# current library and a variant (RANSAC_AMD_LIB), and a kernel trace of the current build.
#   bash tools/gpu_grid_check.sh <variant.so>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/grid; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid_napsac.py tests/test_gpu_napsac_lo.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in ransac_amd/libransac_amd.so $1; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/cfg5_split.py 20 > $O/split.txt 2>&1 || { tail -3 $O/split.txt; exit 1; }
    echo "$lib: $(tail -1 $O/split.txt)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/tr -o run --output-format csv -- python3 tools/cfg5_split.py 5 > /dev/null 2> $O/tr.err || exit $?
