#!/bin/bash
# cfg5 evidence: the default cfg5 bench line, then a rocprofv3 kernel trace of a shorter run.
# Usage (on the GPU box via gpurun): bash tools/gpu_cfg5.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-cfg5}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cfg5 --cpu-seconds 0 "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; cat gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 bench.py --cfg5 --cpu-seconds 0 --steps 20 --warmup 2 "$@" > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_prof.err; exit $rc; }
python3 - "$TAG" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob("gpurun_out/%s_prof/**/*kernel_stats.csv" % tag, recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-44s %6s %9.1f us avg %8.2f ms" % (r["Name"][:44], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
