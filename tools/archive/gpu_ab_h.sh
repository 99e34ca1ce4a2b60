#!/bin/bash
# Same-box A/B of library variants on the default (cfg2) bench line, interleaved, 3 rounds.
# usage (gpurun): bash tools/gpu_ab_h.sh <tag> <variant.so>...   (the current build is always first)
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2 3; do
  for lib in ransac_amd/libransac_amd.so "$@"; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 180 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 > $O/ab.log 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%-34s %8.2f M/s ms/step %.4f score %.4f parity %s' % ('$lib', d['value']/1e6, d['ms_per_step'], r.get('kernel_ms') or 0, d['parity'].get('scores_bit_equal')))"
  done
done
