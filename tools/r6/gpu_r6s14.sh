#!/bin/bash
# head with the one-chain sums on the split segment kernel (default): whole GPU suite, smoke, the
# cfg5 / cfg3-exact lines against USAC_SEQ1_CPL=0 interleaved, bench.py with no flags
set -o pipefail
O=gpurun_out/r6s14; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  for v in 0 d; do
    if [ $v = d ]; then E=""; else E="USAC_SEQ1_CPL=$v"; fi
    env $E timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_c${v}_$r.json 2> $O/cfg5_c${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_c${v}_$r.json'));print('cfg5 seq1=$v', d['ms_per_step'], all(d['parity'].values()))"
    env $E timeout -k 10 200 python -u bench.py --sprt-exact --cpu-seconds 0 > $O/cfg3x_c${v}_$r.json 2> $O/cfg3x_c${v}_$r.err || { echo "cfg3x $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg3x_c${v}_$r.json'));print('cfg3x seq1=$v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('cfg2', d['value'], d['ms_per_step'], d['parity']['ok'])"
timeout -k 10 400 python -u bench.py --cfg5 > $O/cfg5_line.json 2> $O/cfg5_line.err || { echo "cfg5 line failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg5_line.json'));print('cfg5 line', d['ms_per_step'], d['roofline'].get('kernel'), all(d['parity'].values()), d['cpu_baseline']['value'])"
