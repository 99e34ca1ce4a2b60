#!/bin/bash
# e16 drain rounds without per-round barriers ("nosync") vs with ("prev"): tests, phase, cfg4 lines
set -o pipefail
O=gpurun_out/r6qq; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_e16.py tests/test_gpu_essential.py tests/test_gpu_mfma_concurrency.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in prev nosync; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 100 python -u tools/e_phase.py > $O/phase_$v.log 2>&1 || { echo "phase failed"; exit 1; }
echo $v; head -1 $O/phase_$v.log
done
for r in 1 2; do for v in prev nosync; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --estimator essential --steps 30 --warmup 5 --cpu-seconds 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
done; done
