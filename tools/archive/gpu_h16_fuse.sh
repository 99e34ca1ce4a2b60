#!/bin/bash
# The matrix-core scorer's rows written by the solver (default) against k_h16_rows after the solve
# (USAC_H16_FUSE=0): the h16 / parity GPU tests, then interleaved cfg2 lines (100 steps) and a kernel
# trace.  Usage (GPU box): bash tools/gpu_h16_fuse.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-fuse}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_h16.py tests/test_gpu_parity.py tests/test_gpu_edge.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $O/tests.log | head; exit 1; }
for v in "USAC_H16_DEFER=0" "USAC_H16_DEFER=1" "USAC_H16_DEFER=0" "USAC_H16_DEFER=1" "USAC_H16_DEFER=0" "USAC_H16_DEFER=1"; do
  env $v timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '%.1f M hyp/s ms/step %.4f parity %s' % (d['value']/1e6, d['ms_per_step'], d['parity']['ok']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --pipeline 1 > $O/trace.json 2> $O/trace.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
cut -c1-150 $O/trace/run_kernel_stats.csv | head -8
