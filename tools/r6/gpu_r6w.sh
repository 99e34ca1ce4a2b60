#!/bin/bash
# k_e5_roots without the end-value LDS array: tests, phase split, cfg4 lines vs the previous build
set -o pipefail
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_essential.py tests/test_gpu_e5_rpoly.py tests/test_gpu_e16.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in prev cur; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 100 python -u tools/e_phase.py > $O/phase_$v.log 2>&1 || { echo "phase failed"; exit 1; }
echo $v; head -1 $O/phase_$v.log
done
for r in 1 2; do for v in prev cur; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --estimator essential --steps 30 --warmup 5 --cpu-seconds 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
done; done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/$O/trace -o run --output-format csv -- python3 bench.py --estimator essential --steps 10 --warmup 2 --cpu-seconds 0 --pipeline 1 > $O/trace_bench.json 2> $O/trace.err || { echo "trace failed"; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r6w/trace/run_kernel_stats.csv')))
for r in rows[:12]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
