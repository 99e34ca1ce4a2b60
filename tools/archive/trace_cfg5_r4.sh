#!/bin/bash
# cfg5 kernel trace (rocprofv3 --kernel-trace) for the LO-stage timeline and inter-kernel gaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/cfg5_trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O -o run --output-format csv -- \
    python3 bench.py --cfg5 --steps 20 --warmup 3 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 tools/trace_gaps.py $O/run_kernel_trace.csv > $O/gaps.json && cat $O/gaps.json
