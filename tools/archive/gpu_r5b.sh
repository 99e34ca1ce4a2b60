#!/bin/bash
# every -m gpu test on the h16 default, the default bench line, and the h10k PMC profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5b}; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_cfg2.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$O/bench_cfg2.json').read().strip().splitlines()[-1]); r=d['roofline']
print('cfg2 %.1f M hyp/s ms/step %.4f frac %s parity %s cpu %s' % (d['value']/1e6, d['ms_per_step'], r.get('frac'), d['parity']['ok'], d.get('cpu_baseline',{}).get('value')))"
timeout -k 10 300 python bench.py --estimator fundamental > $O/bench_fundamental.json 2> $O/bench_fundamental.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_fundamental.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$O/bench_fundamental.json').read().strip().splitlines()[-1]); c=d['cpu_baseline']
print('cfg3 %.3g hyp/s mph %s | cpu %.3g (%s cores) mph %s equal %s accepted %s | all %.3g' % (d['value'], d.get('models_per_hypothesis'), c['value'], c['cores'], c.get('models_per_hypothesis'), c.get('decisions_equal'), c.get('sprt_accepted'), c['all_cores']['value']))
print(c['sample'])"
TAG=${1:-r5b} WORKLOADS="h10k" bash tools/profile_round.sh > $O/prof.log 2>&1; rc=$?; tail -3 $O/prof.log; exit $rc
