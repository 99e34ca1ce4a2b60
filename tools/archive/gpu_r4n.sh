#!/bin/bash
# k_tv_combine with 16 chunks' loads in flight: two-view tests, cfg4 and F-full lines against the
# previous kernels_fund build (var_libs/lib_fund0.so), interleaved, and a cfg4 kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_twoview_fast.py \
    tests/test_gpu_essential.py tests/test_gpu_fundamental.py tests/test_gpu_baseline_sizes.py > gpurun_out/r4n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4n_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_combine.txt; : > $O
for r in 1 2 3; do
  for v in fund0 new; do
    if [ $v = new ]; then L=$PWD/ransac_amd/libransac_amd.so; else L=$PWD/ransac_amd/var_libs/lib_$v.so; fi
    for mode in "essential" "fundamental --no-sprt --sampler uniform"; do
      RANSAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --estimator $mode --cpu-seconds 0 > gpurun_out/abc.json \
          2> gpurun_out/abc.err || { tail -5 gpurun_out/abc.err; exit 1; }
      python3 - $v "$mode" >> $O <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abc.json").read().strip().splitlines()[-1])
print("%-6s %-40s %8.2f M hyp/s  ms/step %.4f  parity %s" % (sys.argv[1], sys.argv[2], d["value"] / 1e6,
      d["ms_per_step"], d["parity"]["timed_kernel"]["ok"]))
PY
      tail -1 $O
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/r4n_trace -o run --output-format csv -- \
    python3 bench.py --estimator essential --steps 20 --warmup 3 --cpu-seconds 0 --pipeline 1 > gpurun_out/r4n_trace.json \
    2> gpurun_out/r4n_trace.err || { tail -5 gpurun_out/r4n_trace.err; exit 1; }
grep -h "k_tv_combine\|k_score_f2" gpurun_out/r4n_trace/run_kernel_stats.csv | cut -c1-200
