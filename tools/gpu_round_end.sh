#!/bin/bash
# Round-end evidence on one GPU: every -m gpu test, smoke(), the default bench line (cfg2), the
# cfg3 (batch SPRT and the exact sequential SPRT) / cfg4 / cfg5 lines and a rocprofv3 kernel trace
# (--stats) of the default bench.
# Usage (on the GPU box via gpurun): bash tools/gpu_round_end.sh <tag>; outputs gpurun_out/<tag>/.
set -o pipefail
TAG=${1:-end}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; cat $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err
rc=$?; cat $O/bench_cfg2.json; [ $rc -eq 0 ] || exit $rc
for e in fundamental essential; do
  timeout -k 10 300 python bench.py --estimator $e > $O/bench_$e.json 2> $O/bench_$e.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_$e.err; exit $rc; }
done
timeout -k 10 300 python bench.py --cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_cfg5.err; exit $rc; }
timeout -k 10 300 python bench.py --sprt-exact > $O/bench_cfg3_exact.json 2> $O/bench_cfg3_exact.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_cfg3_exact.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/trace_cfg2 -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 > $O/bench_cfg2_traced.json 2> $O/trace_cfg2.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/trace_cfg2.err; exit $rc; }
python3 - $O <<'EOF'
import json, sys
o = sys.argv[1]
for n in ("cfg2", "fundamental", "cfg3_exact", "essential", "cfg5", "cfg2_traced"):
    d = json.loads(open(f"{o}/bench_{n}.json").read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print("%-12s %12.4g %-10s ms/step %.3f frac %.3f parity %s" % (n, d["value"], d["unit"], d["ms_per_step"],
          r.get("frac") or float("nan"), json.dumps(d.get("parity", {}))[:160]))
EOF
