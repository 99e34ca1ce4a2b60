#!/bin/bash
# k_inl_flags / k_inl_compact with the model, threshold and ok loads in flight together (H^-1 per
# lane): whole GPU suite, then cfg5 / cfg3-exact A/B against the head build (var_libs/lib_base.so)
set -o pipefail
O=gpurun_out/r6s11; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then L=$PWD/ransac_amd/var_libs/lib_base.so; else L=$PWD/ransac_amd/libransac_amd.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_${v}_$r.json 2> $O/cfg5_${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_${v}_$r.json'));print('cfg5 $v', d['ms_per_step'], all(d['parity'].values()))"
    RANSAC_AMD_LIB=$L timeout -k 10 200 python -u bench.py --sprt-exact --cpu-seconds 0 > $O/cfg3x_${v}_$r.json 2> $O/cfg3x_${v}_$r.err || { echo "cfg3x $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg3x_${v}_$r.json'));print('cfg3x $v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base new; do
  if [ $v = base ]; then L=$PWD/ransac_amd/var_libs/lib_base.so; else L=$PWD/ransac_amd/libransac_amd.so; fi
  RANSAC_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_$v -o run --output-format csv -- python3 bench.py --cfg5 --cpu-seconds 0 > $O/prof_$v.json 2> $O/prof_$v.err || { echo "prof $v failed"; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
    if 'k_inl' in r['Name']: print('$v', r['Name'][:36], r['Calls'], round(float(r['AverageNs'])/1e3,2))
PY
done
