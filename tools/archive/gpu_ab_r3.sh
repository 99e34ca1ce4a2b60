#!/bin/bash
# cfg2 same-box A/B of the round-3 head (59bd7b2, extracted and built under ab_r3/) against the
# working tree: the driver's own form (--steps 20 --warmup 5) and the 100-step line, interleaved,
# three rounds.  Usage (GPU box): bash tools/gpu_ab_r3.sh; output gpurun_out/ab_r3.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/ab_r3.txt; : > $O
for r in 1 2 3; do
  for v in r3 head; do
    if [ $v = r3 ]; then D=ab_r3; else D=.; fi
    for s in "20 5" "100 10"; do
      set -- $s
      (cd $D && timeout -k 10 120 python3 bench.py --steps $1 --warmup $2 --cpu-seconds 0) \
          > gpurun_out/ab_${v}_$1.json 2> gpurun_out/ab_${v}_$1.err || { tail -5 gpurun_out/ab_${v}_$1.err; exit 1; }
      python3 - $v $1 >> $O <<'EOF'
import json, sys
v, k = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/ab_{v}_{k}.json").read().strip().splitlines()[-1])
r = d.get("roofline", {})
print("%-5s steps %3s %8.1f M hyp/s  ms/step %.4f  solo score %.4f solve %.4f  in-pipe score %.4f  parity %s" % (
    v, k, d["value"] / 1e6, d["ms_per_step"], r.get("score_kernel_ms", 0), r.get("solve_kernel_ms", 0),
    r.get("kernel_ms_in_pipeline", 0), d["parity"].get("inlier_counts_equal")))
EOF
      tail -1 $O
    done
  done
done
