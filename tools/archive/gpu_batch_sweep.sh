#!/bin/bash
# Batch-size sweep of the throughput lines (cfg2 homography, cfg4 essential): 100-step lines per
# batch size, same box.  Usage (GPU box): bash tools/gpu_batch_sweep.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-sweep}; mkdir -p $O
for e in homography essential; do
  for b in 65536 131072 262144; do
    timeout -k 10 300 python bench.py --estimator $e --batch $b --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$e B=$b %.1f M hyp/s ms/step %.4f parity %s' % (d['value']/1e6, d['ms_per_step'], d['parity']['ok']))"
  done
done
