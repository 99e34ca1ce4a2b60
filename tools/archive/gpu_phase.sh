#!/bin/bash
# Per-phase host timings of full runs (USAC_PROFILE=1: setup / draw / device / sums / replay / LO /
# polish per Ransac::run) for the cfg3 exact and cfg5 lines.  Usage (GPU box): bash tools/gpu_phase.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-phase}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_h16.py tests/test_gpu_fundamental.py tests/test_gpu_plugins.py tests/test_gpu_pool.py tests/test_gpu_loop.py -q --timeout 300 --timeout-method thread > $O/tests_h16.log 2>&1
rc=$?; tail -1 $O/tests_h16.log; [ $rc -eq 0 ] || exit $rc
USAC_PROFILE=1 timeout -k 10 300 python bench.py --sprt-exact --steps 30 --warmup 5 --cpu-seconds 0 > $O/cfg3x.json 2> $O/cfg3x.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/cfg3x.err; exit $rc; }
USAC_PROFILE=1 timeout -k 10 300 python bench.py --cfg5 --steps 30 --warmup 5 --cpu-seconds 0 > $O/cfg5.json 2> $O/cfg5.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/cfg5.err; exit $rc; }
python3 - $O <<'PY'
import re, sys, json, numpy as np
o = sys.argv[1]
for n in ("cfg3x", "cfg5"):
    d = json.loads(open(f"{o}/{n}.json").read().strip().splitlines()[-1])
    rows = [list(map(float, re.findall(r"(?:setup|draw|device|sums|replay|lo|polish) ([0-9.]+)", l)))
            for l in open(f"{o}/{n}.err") if l.startswith("usac_ransac_run ms")]
    a = np.array(rows[-30:])
    print(n, "ms/run %.3f" % d["ms_per_step"], "phases (setup draw device sums replay lo polish):",
          " ".join("%.3f" % v for v in a.mean(0)), "n", len(rows))
PY
if [ -n "${WITH_CFG2:-}" ]; then
  timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/cfg2.json 2> $O/cfg2.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $O/cfg2.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/cfg2.json').read().strip().splitlines()[-1]); print('cfg2 %.1f M hyp/s ms/step %.4f frac %.3f parity %s' % (d['value']/1e6, d['ms_per_step'], d['roofline'].get('frac') or -1, d['parity']['ok']))"
fi
if [ -n "${WITH_POLISH_AB:-}" ]; then
  for g in 2 4 1 2 4; do
    USAC_POLISH_GROUP=$g timeout -k 10 300 python bench.py --sprt-exact --steps 50 --warmup 5 --cpu-seconds 0 > $O/px.json 2> $O/px.err || { tail -5 $O/px.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/px.json').read().strip().splitlines()[-1]); print('polish group $g: cfg3 exact ms/run %.3f' % d['ms_per_step'], all(v for k,v in d['parity'].items() if k.endswith('equal')))"
  done
fi
python3 -c "import json; d=json.loads(open('$O/cfg3x.json').read().strip().splitlines()[-1]); print('cfg3x library ms/run', d['run_stats'].get('library_ms_per_run'))"
