#!/bin/bash
# N = 2 rehearsal of bench.py's multi-rank paths on ONE GPU: `bench.py --gpus 2` starts its own two
# rank processes, which share the device (USAC_BENCH_SAME_DEVICE; the record exchange falls back to
# gloo there -- RCCL refuses two ranks on one device).  Lines: cfg2, cfg3 batch SPRT, cfg4, and the
# hypothesis-sharded cfg5 run; each prints n_gpus, the parity verdicts (every rank's slice, the
# first timed batch's merged record against the oracle over both ranks' samples) and the CPU baseline.
# Usage (GPU box): bash tools/gpu_multi_rehearsal.sh [tag]; outputs gpurun_out/<tag>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-multi}; mkdir -p $O
export USAC_BENCH_SAME_DEVICE=1
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 2 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 - $O/$n.json <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d.get("parity", {})
print("%-14s n_gpus %d  %.4g %s  parity.ok %s  ranks %s  first_timed_batch %s  cpu_baseline %s" % (
    sys.argv[1].split("/")[-1], d["n_gpus"], d["value"], d["unit"], p.get("ok", p),
    (p.get("ranks") or {}).get("ok"), (p.get("first_timed_batch") or {}).get("ok"),
    (d.get("cpu_baseline") or {}).get("value")))
EOF
}
run cfg2 --steps 30 --warmup 5 --cpu-seconds 3
run cfg3 --estimator fundamental --steps 30 --warmup 5 --cpu-seconds 3
run cfg4 --estimator essential --steps 20 --warmup 3 --cpu-seconds 3
run cfg5 --cfg5 --steps 10 --warmup 2 --cpu-seconds 3
