#!/bin/bash
# Round-4 session-2 checks on one box: the seqsum / polish / normalisation GPU tests with the
# split segment kernel, then the cfg5 seq-split A/B (USAC_SEQ_SPLIT 0 / 1), the polish-group A/B
# and the cfg2 scorer library A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_seqsum.py \
    "tests/test_gpu_loop.py::test_polish_groups_identical" "tests/test_gpu_loop.py::test_speculation_on_off_identical" \
    > gpurun_out/r4d_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4d_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_seqsplit.txt; : > $O
for r in 1 2 3; do
  for v in 0 1; do
    USAC_SEQ_SPLIT=$v timeout -k 10 120 python3 bench.py --cfg5 --cpu-seconds 0 > gpurun_out/abs.json \
        2> gpurun_out/abs.err || { tail -5 gpurun_out/abs.err; exit 1; }
    python3 - $v >> $O <<'EOF'
import json, sys
d = json.loads(open("gpurun_out/abs.json").read().strip().splitlines()[-1])
print("split %s cfg5 ms/run %.4f  parity %s" % (sys.argv[1], d["ms_per_step"], d["parity"]))
EOF
    tail -1 $O
  done
done
bash tools/archive/gpu_ab_polish.sh || exit 1
bash tools/archive/gpu_ab_cfg2_libs.sh hf_pair hf_quad hf_defer hf_w8 hf_pair_w8
