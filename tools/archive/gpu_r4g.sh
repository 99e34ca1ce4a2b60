#!/bin/bash
# The guarded essential drain: essential / two-view / cfg4 GPU tests, then the cfg4 bench line
# A/B against the round's previous kernels_fund build (var_libs/lib_base.so), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_twoview_fast.py \
    tests/test_gpu_essential.py tests/test_gpu_baseline_sizes.py -k "essential or cfg4 or twoview" \
    > gpurun_out/r4g_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4g_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_cfg4_guard.txt; : > $O
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then L=$PWD/ransac_amd/var_libs/lib_base.so; else L=$PWD/ransac_amd/libransac_amd.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --estimator essential --cpu-seconds 0 \
        > gpurun_out/abg_$v.json 2> gpurun_out/abg_$v.err || { tail -5 gpurun_out/abg_$v.err; exit 1; }
    python3 - $v >> $O <<'EOF'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/abg_{v}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("%-5s %7.2f M hyp/s  ms/step %.4f  score %.4f  solve %.4f  parity %s" % (
    v, d["value"] / 1e6, d["ms_per_step"], r.get("kernel_ms") or -1, r.get("solve_kernel_ms") or -1,
    json.dumps(d.get("parity", {}))[:300]))
EOF
    tail -1 $O
  done
done
