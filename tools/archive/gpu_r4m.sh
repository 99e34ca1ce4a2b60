#!/bin/bash
# NAPSAC grid CSR read in place from a registered host block: the NAPSAC / grid / LO / sharded GPU
# tests, then cfg5 against the previous usac_api build (var_libs/lib_api1.so), interleaved, with the
# run split (USAC_PROFILE) of the new build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grid_napsac.py \
    tests/test_gpu_napsac_lo.py tests/test_gpu_loop.py tests/test_gpu_sharded_run.py tests/test_gpu_plugins.py \
    tests/test_gpu_graphcut.py > gpurun_out/r4m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4m_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_grid_host.txt; : > $O
for r in 1 2 3; do
  for v in api1 new; do
    if [ $v = new ]; then L=$PWD/ransac_amd/libransac_amd.so; else L=$PWD/ransac_amd/var_libs/lib_$v.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --cfg5 --cpu-seconds 0 > gpurun_out/abg.json \
        2> gpurun_out/abg.err || { tail -5 gpurun_out/abg.err; exit 1; }
    python3 - $v >> $O <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abg.json").read().strip().splitlines()[-1])
print("%-5s cfg5 ms/run %.4f  parity %s" % (sys.argv[1], d["ms_per_step"], all(
    v for k, v in d["parity"].items() if isinstance(v, bool))))
PY
    tail -1 $O
  done
done
timeout -k 10 120 python3 tools/cfg5_split.py 30 > gpurun_out/r4m_split.txt 2>&1 || true
tail -3 gpurun_out/r4m_split.txt
