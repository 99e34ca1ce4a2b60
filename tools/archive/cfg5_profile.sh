#!/bin/bash
# cfg5 run split (USAC_PROFILE) averaged over 40 runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
USAC_PROFILE=1 timeout -k 10 120 python tools/cfg5_split.py 40 > gpurun_out/prof_out.txt 2> gpurun_out/prof_err.txt || exit 1
python3 - <<'PY'
import re
rows = [l for l in open("gpurun_out/prof_err.txt") if l.startswith("usac_ransac_run ms")][3:]
keys = ["setup", "draw", "device", "sums", "replay", "lo", "polish", "buffers", "neighbours", "lo/gc"]
acc = {k: 0.0 for k in keys}
for l in rows:
    for k in keys:
        m = re.search(r"\b%s ([0-9.]+)" % re.escape(k), l)
        if m: acc[k] += float(m.group(1))
print(" ".join("%s %.3f" % (k, acc[k] / len(rows)) for k in keys))
print(open("gpurun_out/prof_out.txt").read().strip().splitlines()[-1])
print(rows[-1].strip())
PY
