#!/bin/bash
# round 4: the one-submission polish + one-wait SPRT batches: GPU suite, then cfg5 / cfg3-exact lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/pol
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pol/tests.log 2>&1
rc=$?; tail -3 gpurun_out/pol/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --cfg5 --cpu-seconds 0 > gpurun_out/pol/cfg5_$i.json 2> gpurun_out/pol/cfg5_$i.err || exit 1
  timeout -k 10 300 python bench.py --sprt-exact --cpu-seconds 0 > gpurun_out/pol/cfg3x_$i.json 2> gpurun_out/pol/cfg3x_$i.err || exit 1
done
python3 - <<'PY'
import json
for f in ("cfg5_1", "cfg3x_1", "cfg5_2", "cfg3x_2"):
    d = json.loads(open("gpurun_out/pol/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], json.dumps(d["parity"]))
PY
USAC_PROFILE=1 timeout -k 10 120 python bench.py --sprt-exact --cpu-seconds 0 --steps 20 --warmup 2 > /dev/null 2> gpurun_out/pol/cfg3x_split.txt || exit 1
tail -5 gpurun_out/pol/cfg3x_split.txt
