#!/bin/bash
# the quad root kernel: essential GPU tests, then cfg4 stage times with the lane kernel vs the quad
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_essential.py tests/test_gpu_baseline_sizes.py tests/test_gpu_twoview_fast.py tests/test_gpu_edge.py \
    > gpurun_out/e5_quad_tests.log 2>&1; rc=$?; tail -3 gpurun_out/e5_quad_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_e5_quad.jsonl; : > $O
for r in 1 2; do
  USAC_E5_ROOTS=lane CHUNKS=96 timeout -k 10 180 python3 tools/archive/ab_score_e.py | sed 's/^{/{"roots": "lane", /' >> $O || exit 1
  CHUNKS=96 timeout -k 10 180 python3 tools/archive/ab_score_e.py | sed 's/^{/{"roots": "quad", /' >> $O || exit 1
done
cat $O
for rt in lane quad; do
  USAC_E5_ROOTS=$rt timeout -k 10 300 python3 bench.py --estimator essential --cpu-seconds 0 > gpurun_out/e5_bench_$rt.json 2> gpurun_out/e5_bench_$rt.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/e5_bench_$rt.json').read().strip().splitlines()[-1]); print('$rt', d['value']/1e6, d['ms_per_step'], d['parity']['inlier_counts_equal'], d['parity']['timed_kernel']['ok'])"
done
