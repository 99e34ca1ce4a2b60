#!/bin/bash
# polish submission groups A/B (USAC_POLISH_GROUP 1 / 2 / 4): cfg5 and cfg3-exact lines, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
O=gpurun_out/ab_polish.txt; : > $O
for r in 1 2 3; do
  for g in 1 2 4; do
    for mode in cfg5 sprt-exact; do
      USAC_POLISH_GROUP=$g timeout -k 10 120 python3 bench.py --$mode --cpu-seconds 0 > gpurun_out/abp_$mode.json \
          2> gpurun_out/abp_$mode.err || { tail -5 gpurun_out/abp_$mode.err; exit 1; }
      python3 - $g $mode >> $O <<'EOF'
import json, sys
d = json.loads(open(f"gpurun_out/abp_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print("group %s %-10s ms/run %.4f  parity %s" % (sys.argv[1], sys.argv[2], d["ms_per_step"], all(
    v for k, v in d["parity"].items() if isinstance(v, bool))))
EOF
      tail -1 $O
    done
  done
done
