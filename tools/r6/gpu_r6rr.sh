#!/bin/bash
# head check: the whole GPU suite, smoke, long cfg2 / cfg4 lines (stability)
set -o pipefail
O=gpurun_out/r6rr; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 400 --warmup 5 > $O/cfg2_long.json 2> $O/cfg2_long.err || { echo "cfg2 failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg2_long.json'));print('cfg2 400 steps', d['value']/1e6, d['ms_per_step'], d['parity']['ok'])"
timeout -k 10 300 python -u bench.py --estimator essential --steps 200 --warmup 5 > $O/cfg4_long.json 2> $O/cfg4_long.err || { echo "cfg4 failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg4_long.json'));print('cfg4 200 steps', d['value']/1e6, d['ms_per_step'], d['parity']['ok'])"
