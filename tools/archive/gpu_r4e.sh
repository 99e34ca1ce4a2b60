#!/bin/bash
# seqsum tests (staged link loads), then cfg5 kernel traces with the split / interleaved
# segment kernels (USAC_SEQ_SPLIT 1 / 0): per-kernel stats under gpurun_out/r4e_split{0,1}/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_seqsum.py \
    tests/test_gpu_lsq_weighted.py tests/test_gpu_napsac_lo.py > gpurun_out/r4e_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4e_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  USAC_SEQ_SPLIT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/r4e_split$v -o run \
      --output-format csv -- python3 bench.py --cfg5 --steps 24 --warmup 3 --cpu-seconds 0 \
      > gpurun_out/r4e_split$v.json 2> gpurun_out/r4e_split$v.err || { tail -5 gpurun_out/r4e_split$v.err; exit 1; }
  python3 - $v <<'EOF'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob(f"gpurun_out/r4e_split{v}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("k_seq_", "k_gather_psum4", "k_norm_dist", "k_ata_partial", "k_dlt_finish")):
        print("split %s %-28s calls %5s avg %8.2f us" % (v, r["Name"].split("(")[0].replace("void usac::", "")[:28],
                                                     r["Calls"], float(r["AverageNs"]) / 1e3))
EOF
done
