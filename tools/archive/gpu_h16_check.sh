#!/bin/bash
# h16 bring-up on one GPU: the MFMA f16 lane-map check, the h16 GPU tests, then the cfg2 line with
# the matrix-core prefilter scorer against USAC_H16=0 (k_score_hf), interleaved, and a kernel trace.
# Usage (GPU box): bash tools/gpu_h16_check.sh <tag>; outputs gpurun_out/<tag>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-h16}; mkdir -p $O
timeout -k 10 60 tools/ubench/mfma_f16_layout > $O/layout.json 2>&1; rc=$?; cat $O/layout.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_h16.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    USAC_H16=$v timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
    python3 - $O/b_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("h16=%s %8.1f M hyp/s  ms/step %.4f  solo score %.4f solve %.4f  parity %s tk %s ftb %s" % (sys.argv[2], d["value"] / 1e6,
      d["ms_per_step"], r.get("score_kernel_ms", 0), r.get("solve_kernel_ms", 0), d["parity"]["ok"],
      d["parity"]["timed_kernel"]["ok"], d["parity"].get("first_timed_batch", {}).get("ok")))
PY
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $PWD/$O/trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $O/traced.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec head -12 {} \;
