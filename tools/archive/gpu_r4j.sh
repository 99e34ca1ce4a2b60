#!/bin/bash
# The 16-point A^T A block spec and the folded segment passes: every GPU test, then cfg5 lines
# of the 64-point build (var_libs/lib_ata64.so; its parity flags read false: the oracle follows
# the new spec), the new build without the fold (USAC_SEQ_FOLD=0) and with it, interleaved, and a
# cfg5 kernel trace of the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r4j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4j_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab_ata.txt; : > $O
for r in 1 2 3; do
  for v in ata64 nofold new; do
    if [ $v = ata64 ]; then L=$PWD/ransac_amd/var_libs/lib_$v.so; else L=$PWD/ransac_amd/libransac_amd.so; fi
    F=1; [ $v = nofold ] && F=0
    USAC_SEQ_FOLD=$F RANSAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --cfg5 --cpu-seconds 0 > gpurun_out/aba.json \
        2> gpurun_out/aba.err || { tail -5 gpurun_out/aba.err; exit 1; }
    python3 - $v >> $O <<'EOF'
import json, sys
d = json.loads(open("gpurun_out/aba.json").read().strip().splitlines()[-1])
print("%-6s cfg5 ms/run %.4f  parity %s" % (sys.argv[1], d["ms_per_step"], d["parity"]))
EOF
    tail -1 $O
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/r4j_trace -o run --output-format csv -- \
    python3 bench.py --cfg5 --steps 24 --warmup 3 --cpu-seconds 0 > gpurun_out/r4j_trace.json 2> gpurun_out/r4j_trace.err \
    || { tail -5 gpurun_out/r4j_trace.err; exit 1; }
python3 - <<'EOF'
import csv, glob
f = glob.glob("gpurun_out/r4j_trace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("k_seq_", "k_gather_psum4", "k_norm_dist", "k_ata_partial", "k_dlt_finish",
                                    "k_inl_", "k_fit_small")):
        print("%-28s calls %5s avg %8.2f us" % (r["Name"].split("(")[0].replace("void usac::", "")[:28], r["Calls"],
                                                float(r["AverageNs"]) / 1e3))
EOF
