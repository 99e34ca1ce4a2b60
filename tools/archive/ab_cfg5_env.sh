#!/bin/bash
# A/B of an environment switch on the cfg5 bench (same box, interleaved).  usage: ab_cfg5_env.sh VAR
VAR=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for rep in 1 2 3; do
  for val in 0 1; do
    if [ $val = 1 ]; then E="$VAR=1"; else E="USAC_AB_NONE=1"; fi
    env $E timeout -k 10 200 python bench.py --cfg5 --cpu-seconds 0 "$@" > gpurun_out/ab5.log 2>&1 || { tail -3 gpurun_out/ab5.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab5.log').read().strip().splitlines()[-1]); print('%s=%s %.3f ms/run batches %s parity %s' % ('$VAR', '$val', d['ms_per_step'], d['run_stats']['batches'], all(d['parity'].values())))"
  done
done
