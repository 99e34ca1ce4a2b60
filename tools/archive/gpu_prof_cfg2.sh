#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of a short default bench: per-kernel averages.
# usage (gpurun): bash tools/gpu_prof_cfg2.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/tr -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 "$@" > $O/bench_traced.json 2> $O/tr.err || { tail -5 $O/tr.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob("%s/tr/**/*kernel_stats.csv" % sys.argv[1], recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("   %-60s %6s %9.1f us avg %9.1f max" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
