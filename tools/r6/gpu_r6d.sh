#!/bin/bash
set -o pipefail
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_essential.py tests/test_gpu_e16.py tests/test_gpu_baseline_sizes.py -k "essential or cfg4 or e16 or e5" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
timeout -k 10 200 python -u tools/e_phase.py > $O/phase.log 2>&1; echo "phase rc=$?"; cat $O/phase.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o e -- python3 $GRAFT_REPO_ROOT/tools/e_phase.py > /dev/null 2>&1; echo "prof rc=$?"
