#!/bin/bash
set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 60 ./tools/ubench/jt_bench > $O/jt_bench.log 2>&1; echo "jt_bench rc=$?"; cat $O/jt_bench.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_e5_rpoly.py tests/test_gpu_essential.py tests/test_gpu_baseline_sizes.py -k "rpoly or log or essential or cfg4" > $O/tests.log 2>&1; echo "tests rc=$?"; grep -E "PASS|FAIL|Error|passed|failed|differ" $O/tests.log | tail -15
timeout -k 10 200 python -u tools/e_phase.py > $O/phase.log 2>&1; echo "phase rc=$?"; cat $O/phase.log
