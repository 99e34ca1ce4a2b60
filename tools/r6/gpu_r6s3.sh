#!/bin/bash
# psum / norm_dist loads in flight A/B (base = the link-staging commit)
# HEAD build (var_libs/lib_base.so) and the new one interleaved, then a kernel trace of the new
set -o pipefail
O=gpurun_out/r6s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_seqsum.py tests/test_gpu_loop.py tests/test_gpu_napsac_lo.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then L=$PWD/ransac_amd/var_libs/lib_base.so; else L=$PWD/ransac_amd/libransac_amd.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python -u bench.py --cfg5 > $O/cfg5_${v}_$r.json 2> $O/cfg5_${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_${v}_$r.json'));print('$v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --cfg5 > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_cfg5.csv
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$O/kernel_stats_cfg5.csv')))
for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:22]: print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['TotalDurationNs'])/1e3,1))
PY
