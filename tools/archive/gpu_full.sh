#!/bin/bash
# Full GPU check: every -m gpu test, smoke(), then the default bench line (N = 1).
# Usage (on the GPU box via gpurun): bash tools/gpu_full.sh <tag>
set -o pipefail
TAG=${1:-full}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; cat gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; cat gpurun_out/${TAG}_bench.json; exit $rc
