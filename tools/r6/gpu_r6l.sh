#!/bin/bash
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_h16.py tests/test_gpu_mfma_concurrency.py tests/test_gpu_loop.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_h.json 2> $O/bench_h.err || { echo "bench failed"; tail $O/bench_h.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_h.json'));print(d['value']/1e6, d['ms_per_step'], d['roofline'])"
