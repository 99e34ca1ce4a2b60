#!/bin/bash
# A/B of environment settings on cfg5 wall time per run: ab_env_run.sh R "ENV=A" "ENV=B" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abenv; mkdir -p $O
R=$1; shift
for rep in $(seq $R); do
  for env in "$@"; do
    env $env USAC_PROFILE=1 timeout -k 10 120 python tools/cfg5_split.py 40 > $O/out.txt 2> $O/err.txt || exit 1
    python3 -c "
import re
l=[x for x in open('$O/err.txt') if x.startswith('usac_ransac_run ms')][3:]
lo=[float(re.search(r' lo ([0-9.]+)',x).group(1)) for x in l]
print('%-24s lo %.3f  %s'%('$env',sum(lo)/len(lo),open('$O/out.txt').read().strip().splitlines()[-1]))"
  done
done
