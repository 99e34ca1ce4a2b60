#!/bin/bash
# Same-box A/B of cfg5 runs with the USAC_PROFILE split (lo / total per run), alternating the
# current library and a variant R times.   bash tools/ab_cfg5_lo.sh <variant.so> [R] [runs]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ablo; mkdir -p $O
V=$1; R=${2:-5}; N=${3:-30}
for rep in $(seq $R); do
  for lib in ransac_amd/libransac_amd.so $V; do
    USAC_PROFILE=1 RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/cfg5_split.py $N > $O/out.txt 2> $O/err.txt || { tail -3 $O/err.txt; exit 1; }
    python3 - "$lib" $O <<'PY'
import re, sys
lines = [l for l in open(sys.argv[2] + "/err.txt") if l.startswith("usac_ransac_run ms")][3:]
lo = [float(re.search(r" lo ([0-9.]+)", l).group(1)) for l in lines]
tot = sum(float(x) for x in re.findall(r"(?:setup|draw|device|sums|replay|lo|polish) ([0-9.]+)", lines[0])) if lines else 0
run = open(sys.argv[2] + "/out.txt").read().strip().splitlines()[-1]
print("%-40s lo %.3f ms  %s" % (sys.argv[1], sum(lo) / len(lo), run))
PY
  done
done
