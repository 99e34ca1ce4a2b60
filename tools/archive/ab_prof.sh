#!/bin/bash
# per-kernel average durations (rocprofv3 --kernel-trace --stats) of the default bench for
# several library builds: ab_prof.sh <lib.so>... [-- bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ $# -gt 0 ] && shift
mkdir -p gpurun_out/abprof
for lib in "${libs[@]}"; do
  name=$(basename $lib .so)
  export RANSAC_AMD_LIB=$PWD/$lib
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof/$name -o run --output-format csv -- \
      python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/abprof/$name.json 2> gpurun_out/abprof/$name.err || { tail -5 gpurun_out/abprof/$name.err; exit 1; }
  python3 - "$name" <<'PY'
import csv, glob, json, sys
name = sys.argv[1]
d = json.loads(open("gpurun_out/abprof/%s.json" % name).read().strip().splitlines()[-1])
print("== %s  %.2f M/s  ms/step %.4f  parity %s" % (name, d["value"] / 1e6, d["ms_per_step"], d.get("parity", {}).get("scores_bit_equal")))
f = glob.glob("gpurun_out/abprof/%s/**/*kernel_stats.csv" % name, recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("   %-48s %5s %9.1f us" % (r["Name"][:48], r["Calls"], float(r["AverageNs"]) / 1000))
PY
done
