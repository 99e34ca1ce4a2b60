#!/bin/bash
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_e5_rpoly.py tests/test_gpu_baseline_sizes.py -k "rpoly or log or cfg4" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/tests.log
for b in 192 320 640; do USAC_E5_BUDGET=$b timeout -k 10 100 python -u tools/e_phase.py > $O/phase_$b.log 2>&1; echo "budget $b rc=$?"; head -1 $O/phase_$b.log; done
for q in 4 8; do GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 0 --pipeline 8 > $O/bench_q$q.json 2> $O/bench_q$q.err; echo "queues $q rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_q$q.json'));print(d['value']/1e6, d['ms_per_step'])"; done
