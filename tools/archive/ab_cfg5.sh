#!/bin/bash
# A/B of library builds on cfg5 runs: per build the run wall split and the LO kernels' average
# durations (rocprofv3 --kernel-trace --stats).  ab_cfg5.sh <lib.so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abc5
for lib in "$@"; do
  name=$(basename $lib .so)
  export RANSAC_AMD_LIB=$PWD/$lib
  timeout -k 10 120 python tools/cfg5_split.py 20 > gpurun_out/abc5/$name.txt 2>&1 || { tail -3 gpurun_out/abc5/$name.txt; exit 1; }
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/abc5/$name -o run --output-format csv -- \
      python3 tools/cfg5_split.py 10 > /dev/null 2> gpurun_out/abc5/$name.err || { tail -3 gpurun_out/abc5/$name.err; exit 1; }
  echo "== $name: $(tail -1 gpurun_out/abc5/$name.txt)"
  python3 - $name <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/abc5/%s/**/*kernel_stats.csv" % sys.argv[1], recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r["TotalDurationNs"]) > 2e6:
        print("   %-44s %6s %8.1f us" % (r["Name"][:44], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
