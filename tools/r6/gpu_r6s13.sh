#!/bin/bash
# one-chain sums (Σerr) through the split segment kernel (USAC_SEQ1_CPL 1 / 2 / 4) vs k_seq_seg:
# seqsum / loop tests under each, cfg5 and cfg3-exact lines interleaved, kernel stats per variant
set -o pipefail
O=gpurun_out/r6s13; mkdir -p $O
for v in 1 2 4; do
  USAC_SEQ1_CPL=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_seqsum.py tests/test_gpu_loop.py tests/test_gpu_napsac_lo.py > $O/tests_c$v.log 2>&1 || { echo "tests $v failed"; tail -5 $O/tests_c$v.log; exit 1; }
  echo "tests seq1_cpl=$v: $(tail -1 $O/tests_c$v.log)"
done
for r in 1 2 3; do
  for v in 0 1 2 4; do
    USAC_SEQ1_CPL=$v timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_c${v}_$r.json 2> $O/cfg5_c${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_c${v}_$r.json'));print('cfg5 seq1_cpl=$v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
for v in 0 2; do
  USAC_SEQ1_CPL=$v timeout -k 10 200 python -u bench.py --sprt-exact --cpu-seconds 0 > $O/cfg3x_c${v}.json 2> $O/cfg3x_c${v}.err || { echo "cfg3x $v failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cfg3x_c${v}.json'));print('cfg3x seq1_cpl=$v', d['ms_per_step'], all(d['parity'].values()))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1 2 4; do
  USAC_SEQ1_CPL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_c$v -o run --output-format csv -- python3 bench.py --cfg5 --cpu-seconds 0 > $O/prof_c$v.json 2> $O/prof_c$v.err || { echo "prof $v failed"; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open('$O/prof_c$v/run_kernel_stats.csv')):
    if 'seq_seg' in r['Name']: print('seq1_cpl=$v', r['Name'][:44], r['Calls'], round(float(r['AverageNs'])/1e3,2))
PY
done
