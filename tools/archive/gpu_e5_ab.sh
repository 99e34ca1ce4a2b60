#!/bin/bash
# cfg4 check: the essential GPU tests, the cfg4 line (twice) and a kernel trace of one batch at a
# time.  Round 5 ran it as an A/B of 5-point solver variants (an LDS determinant with a pivot
# permutation, a 16-lane root isolation): all slower, not kept -- profiles/r5/e5_ab.txt.
# Usage (GPU box): bash tools/gpu_e5_ab.sh <tag>; outputs gpurun_out/<tag>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-e5ab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_essential.py tests/test_gpu_baseline_sizes.py -q -k "essential or cfg4 or e5" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -le 1 ] || exit $rc; grep -q failed $O/tests.log && { grep -E "^FAILED|Error" $O/tests.log | head; exit 1; }
for v in "run=1" "run=2"; do
  env $v timeout -k 10 300 python bench.py --estimator essential --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '%.1f M hyp/s ms/step %.4f parity %s' % (d['value']/1e6, d['ms_per_step'], d['parity']['ok']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/trace -o run --output-format csv -- \
    python3 bench.py --estimator essential --steps 20 --warmup 3 --cpu-seconds 0 --pipeline 1 > $O/trace.json 2> $O/trace.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
grep -h "k_e5" $O/trace/run_kernel_stats.csv | cut -c1-160
