#!/bin/bash
# cfg2 bench-line A/B over library builds: base and var_libs/lib_<v>.so, interleaved, 2 rounds;
# plus the solo score-kernel times (ab_score_h.py).  Usage: gpu_ab_cfg2_libs.sh <v>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
O=gpurun_out/ab_cfg2_libs.txt; : > $O
for r in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=$PWD/ransac_amd/libransac_amd.so; else L=$PWD/ransac_amd/var_libs/lib_$v.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 \
        > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
    RANSAC_AMD_LIB=$L timeout -k 10 120 python3 tools/archive/ab_score_h.py > gpurun_out/ab_$v.solo || exit 1
    python3 - $v >> $O <<'EOF'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{v}.json").read().strip().splitlines()[-1])
s = json.loads(open(f"gpurun_out/ab_{v}.solo").read().strip().splitlines()[-1])
print("%-12s %8.1f M hyp/s  ms/step %.4f  parity %s  solo score %.4f (min %.4f) solve %.4f" % (
    v, d["value"] / 1e6, d["ms_per_step"], d["parity"].get("inlier_counts_equal"), s["score_ms_med"],
    s["score_ms_min"], s["solve_ms_med"]))
EOF
    tail -1 $O
  done
done
