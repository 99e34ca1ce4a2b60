#!/bin/bash
# round 6: the h16 race diagnostic, the essential GPU tests (rpoly order), the cfg4 line + its kernel trace
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 300 ./tools/h16_race > gpurun_out/r6a/race.log 2>&1; echo "race rc=$?"
tail -30 gpurun_out/r6a/race.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_essential.py tests/test_gpu_e16.py tests/test_gpu_baseline_sizes.py -k "essential or cfg4 or e5 or e16" > gpurun_out/r6a/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/r6a/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 2 > gpurun_out/r6a/bench_e.json 2> gpurun_out/r6a/bench_e.err; echo "bench rc=$?"; tail -c 1500 gpurun_out/r6a/bench_e.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6a/prof -o e -- python3 $GRAFT_REPO_ROOT/bench.py --estimator essential --steps 5 --warmup 2 --cpu-seconds 0 > /dev/null 2>&1; echo "prof rc=$?"
