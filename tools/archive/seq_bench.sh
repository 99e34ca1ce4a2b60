#!/bin/bash
# Σerr chain micro-bench under rocprofv3 (tools/seq_bench.py): per-kernel times of one
# get_inliers (flags, compaction, the three seqsum kernels) at N elements.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
N=${1:-20000}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/seqb -o run --output-format csv -- \
    python3 tools/seq_bench.py $N 200 || exit 1
f=$(find gpurun_out/seqb -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')): print('%-50s %6s %8.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))"
