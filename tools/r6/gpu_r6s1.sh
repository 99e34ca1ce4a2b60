#!/bin/bash
# seqsum link staging A/B: the seqsum / loop tests on the new build, then cfg5 lines of the
# HEAD build (var_libs/lib_base.so) and the new one interleaved, then a kernel trace of the new
set -o pipefail
O=gpurun_out/r6s1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_seqsum.py tests/test_gpu_loop.py tests/test_gpu_napsac_lo.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then L=$PWD/ransac_amd/var_libs/lib_base.so; else L=$PWD/ransac_amd/libransac_amd.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python -u bench.py --cfg5 > $O/cfg5_${v}_$r.json 2> $O/cfg5_${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_${v}_$r.json'));print('$v', d['value'], d['ms_per_step'], d['parity']['ok'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --cfg5 > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_cfg5.csv
python3 - <<EOF
import csv
for r in csv.DictReader(open('$O/kernel_stats_cfg5.csv')):
    if 'seq' in r['Name'] or 'inl' in r['Name']: print(r['Name'][:50], r['Calls'], r['AverageNs'])
EOF
