#!/bin/bash
# PROSAC best updates with the inlier list copied in the scoring submission: the PROSAC / SPRT
# loop tests, then the cfg3-exact line against the previous usac_api build (var_libs/lib_api0.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_loop.py \
    tests/test_gpu_baseline_sizes.py tests/test_gpu_plugins.py > gpurun_out/r4l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4l_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_prosac_list.txt; : > $O
for r in 1 2 3; do
  for v in api0 new; do
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
# cfg2 against the build of the round's first round-end run (d8df98a, var_libs/lib_r4b.so): a
# regression check of the default line (box-to-box spread is +-10 %, so same box, interleaved)
O=gpurun_out/ab_cfg2_r4b.txt; : > $O
for r in 1 2 3; do
  for v in r4b new; do
    if [ $v = new ]; then L=$PWD/ransac_amd/libransac_amd.so; else L=$PWD/ransac_amd/var_libs/lib_$v.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --cpu-seconds 0 > gpurun_out/abr.json \
        2> gpurun_out/abr.err || { tail -5 gpurun_out/abr.err; exit 1; }
    python3 - $v >> $O <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abr.json").read().strip().splitlines()[-1])
print("%-4s cfg2 %7.2f M hyp/s  ms/step %.4f  parity %s" % (sys.argv[1], d["value"] / 1e6, d["ms_per_step"],
      d["parity"]["timed_kernel"]["ok"]))
PY
    tail -1 $O
  done
done
