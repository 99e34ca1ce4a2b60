#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench.  Stops at the first step that
# crashes, aborts or times out (exit codes other than 0 and pytest's 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-20}
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "== pytest -m gpu rc=$rc"; tail -n 40 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "== smoke rc=$rc"; tail -n 20 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "== bench rc=$rc"; cat gpurun_out/bench.json; tail -n 20 gpurun_out/bench.err
exit $rc
