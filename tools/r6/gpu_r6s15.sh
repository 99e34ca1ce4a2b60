#!/bin/bash
# final head check (after the USAC_SEQ1_CPL switch went in, default off) in the driver forms
set -o pipefail
O=gpurun_out/r6s15; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['metric'], d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['ok'], d['cpu_baseline']['value'])"
