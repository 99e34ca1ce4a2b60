#!/bin/bash
# cfg4 solve-stage kernel times vs batch size (rocprofv3 kernel trace, one batch in flight).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/e5_batch; mkdir -p $O
for B in 65536 262144; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $PWD/$O/b$B -o run --output-format csv -- \
      python3 bench.py --estimator essential --batch $B --steps 10 --warmup 2 --cpu-seconds 0 --pipeline 1 \
      > $O/b$B.json 2> $O/b$B.err || { tail -5 $O/b$B.err; exit 1; }
  python3 tools/summarize_profile.py $O/b$B e5b$B 50000 $B $O/sum > /dev/null || exit 1
done
python3 - <<'PY'
import json
for B in (65536, 262144):
    d = json.load(open("gpurun_out/e5_batch/sum/e5b%d_summary.json" % B))
    for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["trace"]["avg_ns"])[:8]:
        print(B, "%10.1f us" % (v["trace"]["avg_ns"] / 1e3), k[:70])
PY
