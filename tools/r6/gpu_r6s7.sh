#!/bin/bash
# the fit's finish in its last A^T A workgroup (USAC_FIT_FUSED_FINISH, default on): whole GPU
# suite + smoke, then cfg5 / cfg3-exact lines with it off and on, interleaved, on one box
set -o pipefail
O=gpurun_out/r6s7; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
  for v in 0 1; do
    USAC_FIT_FUSED_FINISH=$v timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_f${v}_$r.json 2> $O/cfg5_f${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_f${v}_$r.json'));print('cfg5 fused=$v', d['ms_per_step'], all(d['parity'].values()))"
    USAC_FIT_FUSED_FINISH=$v timeout -k 10 200 python -u bench.py --sprt-exact --cpu-seconds 0 > $O/cfg3x_f${v}_$r.json 2> $O/cfg3x_f${v}_$r.err || { echo "cfg3x $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg3x_f${v}_$r.json'));print('cfg3x fused=$v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
