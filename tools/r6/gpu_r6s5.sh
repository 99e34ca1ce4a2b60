#!/bin/bash
# after the seqsum load fixes: whole GPU suite + smoke; cfg3 exact and cfg5 lines of the round's
# earlier build (var_libs/lib_base.so: seqsum / nonmin kernels before the fixes) and the head,
# interleaved; the cfg5 profile (trace + PMC passes) for bench.py's cfg5 roofline
set -o pipefail
O=gpurun_out/r6s5; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then L=$PWD/ransac_amd/var_libs/lib_base.so; else L=$PWD/ransac_amd/libransac_amd.so; fi
    RANSAC_AMD_LIB=$L timeout -k 10 200 python -u bench.py --sprt-exact --cpu-seconds 0 > $O/cfg3x_${v}_$r.json 2> $O/cfg3x_${v}_$r.err || { echo "cfg3x $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg3x_${v}_$r.json'));print('cfg3x $v', d['ms_per_step'], d['value'])"
    RANSAC_AMD_LIB=$L timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_${v}_$r.json 2> $O/cfg5_${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_${v}_$r.json'));print('cfg5 $v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
TAG=r6t WORKLOADS="cfg5" timeout -k 10 900 bash tools/profile_round.sh > $O/profile.log 2>&1 || { echo "profile failed"; tail -5 $O/profile.log; exit 1; }
mkdir -p $O/summaries && cp gpurun_out/prof_r6t/summaries/* $O/summaries/ && ls $O/summaries
