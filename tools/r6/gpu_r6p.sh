#!/bin/bash
# essential root-order kernels on a CU-masked stream: tests, cfg4 lines by mask size
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_e16.py tests/test_gpu_essential.py tests/test_gpu_e5_rpoly.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 0 32 16 64; do
USAC_E5_THIN_CUS=$c USAC_E16=1 timeout -k 10 200 python -u bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_$c.json 2> $O/b_$c.err || { echo "bench failed"; tail -5 $O/b_$c.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_$c.json'));print('cus $c', d['value']/1e6, d['ms_per_step'], d.get('parity',{}).get('ok'))"
done
