#!/bin/bash
# cfg3 batch / pipeline-depth sweep with the guarded drains (two interleaved rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
O=gpurun_out/f_sweep.txt; : > $O
for r in 1 2; do
  for cfg in "65536 3" "131072 3" "262144 3" "262144 2" "524288 2" "131072 2"; do
    set -- $cfg
    timeout -k 10 200 python3 bench.py --estimator fundamental --cpu-seconds 0 --batch $1 --pipeline $2 \
        > gpurun_out/fs.json 2> gpurun_out/fs.err || { tail -5 gpurun_out/fs.err; exit 1; }
    python3 - $1 $2 >> $O <<'EOF'
import json, sys
d = json.loads(open("gpurun_out/fs.json").read().strip().splitlines()[-1])
print("B %6s pipe %s  %7.2f M hyp/s  ms/step %.4f  parity %s" % (sys.argv[1], sys.argv[2], d["value"] / 1e6,
      d["ms_per_step"], d.get("parity", {}).get("timed_kernel", {}).get("ok")))
EOF
    tail -1 $O
  done
done
