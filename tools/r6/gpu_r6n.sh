#!/bin/bash
# early-stop rpoly order: essential parity tests, phase split, cfg4 bench (e16 on and off)
set -o pipefail
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_essential.py tests/test_gpu_e5_rpoly.py tests/test_gpu_e16.py tests/test_gpu_twoview_fast.py tests/test_gpu_baseline_sizes.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 100 python -u tools/e_phase.py > $O/phase.log 2>&1; echo "phase rc=$?"; cat $O/phase.log
for e in 1 0; do
USAC_E16=$e timeout -k 10 200 python -u bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_e16_$e.json 2> $O/bench_e16_$e.err || { echo "bench failed"; tail -5 $O/bench_e16_$e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_e16_$e.json'));print('e16=$e', d['value']/1e6, d['ms_per_step'], d.get('parity',{}).get('ok'))"
done
