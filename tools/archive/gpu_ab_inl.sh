#!/bin/bash
# inlier-kernel change check: every GPU test that scores inlier lists, then the LO-split A/B
#   bash tools/gpu_ab_inl.sh <variant.so> [R]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab_inl_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_inl_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_cfg5_lo.sh $1 ${2:-6} 40 > gpurun_out/ab_lo.txt || exit 1
python3 - <<'PY'
import re, statistics as st
a = {"new": [], "old": []}; r = {"new": [], "old": []}
for l in open("gpurun_out/ab_lo.txt"):
    m = re.search(r"lo ([0-9.]+) ms.*run ([0-9.]+)", l)
    if not m: continue
    k = "new" if "libransac_amd.so" in l.split()[0] else "old"
    a[k].append(float(m.group(1))); r[k].append(float(m.group(2)))
for k in a:
    print(k, "lo mean %.3f median %.3f   run mean %.3f median %.3f" % (st.mean(a[k]), st.median(a[k]), st.mean(r[k]), st.median(r[k])))
PY
