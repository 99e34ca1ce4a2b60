#!/bin/bash
# cfg2 A/B of the h16 scorer variants (USAC_H16_NA 2 / 4, USAC_H16_CHUNKS) against USAC_H16=0, two
# interleaved rounds, then a rocprofv3 kernel trace of one batch at a time (--pipeline 1: the
# kernels' solo durations).  Usage (GPU box): bash tools/gpu_h16_ab.sh <tag> ["ENV=.. ENV=.." ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-h16ab}; shift
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_h16.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VARS=("USAC_H16=0" "$@")
for r in 1 2; do
  k=0
  for v in "${VARS[@]}"; do
    env $v timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 > $O/b_$k.json 2> $O/b_$k.err || { tail -5 $O/b_$k.err; exit 1; }
    python3 - $O/b_$k.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-40s %8.1f M hyp/s  ms/step %.4f  solo score %.4f solve %.4f  parity %s" % (sys.argv[2], d["value"] / 1e6,
      d["ms_per_step"], r.get("score_kernel_ms", 0), r.get("solve_kernel_ms", 0), d["parity"]["ok"]))
PY
    k=$((k+1))
  done
done
env ${VARS[1]:-USAC_H16=1} timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $PWD/$O/trace -o run --output-format csv -- \
    python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 --pipeline 1 > $O/traced.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec head -10 {} \; | cut -c1-60,180-260
