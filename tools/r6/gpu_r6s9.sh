#!/bin/bash
# round-6 head (seq segment kernel: 2 candidates per lane for the fp32 chains): whole GPU suite,
# smoke, cfg5 / cfg3-exact A/B against USAC_SEQ_CPL=1, every default bench line, cfg5 kernel stats
set -o pipefail
O=gpurun_out/r6s9; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
  for v in 1 d; do
    if [ $v = d ]; then E=""; else E="USAC_SEQ_CPL=$v"; fi
    env $E timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_c${v}_$r.json 2> $O/cfg5_c${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_c${v}_$r.json'));print('cfg5 cpl=$v', d['ms_per_step'], all(d['parity'].values()))"
    env $E timeout -k 10 200 python -u bench.py --sprt-exact --cpu-seconds 0 > $O/cfg3x_c${v}_$r.json 2> $O/cfg3x_c${v}_$r.err || { echo "cfg3x $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg3x_c${v}_$r.json'));print('cfg3x cpl=$v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
line() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d['roofline'];print('$n', d['value'], d['ms_per_step'], r.get('kernel'), r.get('frac'), d.get('cpu_baseline',{}).get('value'), d.get('parity',{}).get('ok', d.get('parity')))"
}
line cfg2 --steps 20 --warmup 5
line cfg3 --estimator fundamental --steps 20 --warmup 5
line cfg3x --sprt-exact --steps 20 --warmup 3
line cfg4 --estimator essential --steps 20 --warmup 5
line cfg5 --cfg5
line cfg5_s20 --cfg5 --steps 20 --warmup 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_cfg5 -o run --output-format csv -- python3 bench.py --cfg5 --cpu-seconds 0 > $O/prof_cfg5.json 2> $O/prof_cfg5.err || { echo "prof cfg5 failed"; exit 1; }
echo done
