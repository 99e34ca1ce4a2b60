#!/bin/bash
# LO stage events without timestamps (USAC_LO_SYNC_EV) x stage graphs (USAC_LO_GRAPH): cfg5 A/B,
# four variants interleaved, three rounds; the loop tests first
set -o pipefail
O=gpurun_out/r6s4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_seqsum.py tests/test_gpu_loop.py tests/test_gpu_napsac_lo.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR| passed| failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in s0g0 s1g0 s1g1 s0g1; do
    S=${v:1:1}; G=${v:3:1}
    USAC_LO_SYNC_EV=$S USAC_LO_GRAPH=$G timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_${v}_$r.json 2> $O/cfg5_${v}_$r.err || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_${v}_$r.json'));print('$v', d['ms_per_step'], all(d['parity'].values()))"
  done
done
