#!/bin/bash
# the h16 batch argmax at 256 hypotheses per workgroup ("amx") vs 2048 ("cur")
set -o pipefail
O=gpurun_out/r6ff; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_loop.py tests/test_gpu_h16.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in cur amx; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 > $O/h_${v}_$r.json 2> $O/h_${v}_$r.err || { echo "bench failed"; tail -5 $O/h_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/h_${v}_$r.json'));print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],4))"
done; done
cat /proc/loadavg
