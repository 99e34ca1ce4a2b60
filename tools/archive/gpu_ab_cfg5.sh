#!/bin/bash
# Same-box A/B of cfg5 runs: the given GPU tests on the current library, then cfg5 wall time per
# run (tools/cfg5_split.py, 20 runs) alternating current / variant, and a kernel trace of the
# current build.   bash tools/gpu_ab_cfg5.sh <variant.so> [test files...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/abc5; mkdir -p $O
V=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread "$@" > $O/tests.log 2>&1; rc=$?
  tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2 3; do
  for lib in ransac_amd/libransac_amd.so $V; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/cfg5_split.py 20 > $O/split.txt 2>&1 || { tail -3 $O/split.txt; exit 1; }
    echo "$lib: $(tail -1 $O/split.txt)"
  done
done
timeout -k 10 300 python bench.py --cfg5 > $O/cfg5.json 2> $O/cfg5.err || { tail -3 $O/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/cfg5.json').read().splitlines()[-1]); print('bench cfg5', d['ms_per_step'], d['parity'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/tr -o run --output-format csv -- python3 tools/cfg5_split.py 5 > /dev/null 2> $O/tr.err || exit $?
