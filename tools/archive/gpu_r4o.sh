#!/bin/bash
# The PROSAC termination scan from the sorted inlier list with lazy maximality updates: the PROSAC / SPRT
# loop tests, then the cfg3-exact line against the previous usac_api build (var_libs/lib_api2.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_loop.py \
    tests/test_gpu_baseline_sizes.py tests/test_gpu_plugins.py tests/test_gpu_cpp_consumer.py tests/test_gpu_reference_statistics.py > gpurun_out/r4o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4o_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_prosac_scan.txt; : > $O
for r in 1 2 3; do
  for v in api2 new; do
    if [ $v = new ]; then L=$PWD/ransac_amd/libransac_amd.so; else L=$PWD/ransac_amd/var_libs/lib_$v.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --sprt-exact --cpu-seconds 0 > gpurun_out/abl.json \
        2> gpurun_out/abl.err || { tail -5 gpurun_out/abl.err; exit 1; }
    python3 - $v >> $O <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abl.json").read().strip().splitlines()[-1])
print("%-5s cfg3 exact ms/run %.4f  parity %s" % (sys.argv[1], d["ms_per_step"], all(
    v for k, v in d["parity"].items() if isinstance(v, bool))))
PY
    tail -1 $O
  done
done
