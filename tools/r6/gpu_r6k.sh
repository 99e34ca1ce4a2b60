#!/bin/bash
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_e16.py tests/test_gpu_mfma_concurrency.py > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
timeout -k 10 100 python -u tools/e_phase.py > $O/phase.log 2>&1; echo "phase rc=$?"; cat $O/phase.log
USAC_E16=1 timeout -k 10 200 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_e16.json 2> $O/bench_e16.err; echo "e16 rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_e16.json'));print(d['value']/1e6, d['ms_per_step'])"
