#!/bin/bash
# round 6: race diagnostic after the packed-fp32 removal, the whole GPU suite, cfg4 + cfg2 lines, cfg4 trace
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 ./tools/h16_race > $O/race.log 2>&1; echo "race rc=$?"; grep "^mode" $O/race.log
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -25
timeout -k 10 300 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 2 > $O/bench_e.json 2> $O/bench_e.err; echo "bench_e rc=$?"; head -c 600 $O/bench_e.json; echo
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_h.json 2> $O/bench_h.err; echo "bench_h rc=$?"; head -c 600 $O/bench_h.json; echo
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_e -o e -- python3 $GRAFT_REPO_ROOT/bench.py --estimator essential --steps 5 --warmup 2 --cpu-seconds 0 > /dev/null 2>&1; echo "prof rc=$?"
