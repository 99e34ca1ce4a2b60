#!/bin/bash
# e16 per-lane stacks vs the shared ring (spectral-norm slack in both): tests, phase split, cfg4 lines;
# then a cfg4 kernel trace and the cfg5 profile (trace + PMC passes of bench.py --cfg5 itself)
set -o pipefail
O=gpurun_out/r6o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_e16.py tests/test_gpu_essential.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in e16ring e16stack; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 100 python -u tools/e_phase.py > $O/phase_$v.log 2>&1 || { echo "phase failed"; exit 1; }
echo $v; head -1 $O/phase_$v.log
done
for r in 1 2; do for v in e16ring e16stack; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so USAC_E16=1 timeout -k 10 200 python -u bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', d['value']/1e6, d['ms_per_step'], d.get('parity',{}).get('ok'))"
done; done
USAC_E16=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/e4trace -o run --output-format csv -- \
    python3 bench.py --estimator essential --steps 20 --warmup 3 --cpu-seconds 0 > $O/e4_bench.json 2> $O/e4_trace.err || { echo "e4 trace failed"; tail -5 $O/e4_trace.err; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r6o/e4trace/run_kernel_stats.csv')))
for r in rows[:16]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'][:5])
PY
TAG=r6 WORKLOADS=cfg5 bash tools/profile_round.sh > $O/prof_cfg5.log 2>&1 || { echo "cfg5 profile failed"; tail -20 $O/prof_cfg5.log; exit 1; }
tail -8 $O/prof_cfg5.log
