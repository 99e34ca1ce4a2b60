#!/bin/bash
# Selected GPU tests: bash tools/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/${TAG}.log 2>&1
rc=$?; tail -30 gpurun_out/${TAG}.log; exit $rc
