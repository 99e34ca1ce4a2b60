#!/bin/bash
# cfg5 profile at the head (trace + PMC passes, tools/profile_round.sh) for bench.py's cfg5 roofline
set -o pipefail
O=gpurun_out/r6s10; mkdir -p $O
TAG=r6v WORKLOADS="cfg5" timeout -k 10 900 bash tools/profile_round.sh > $O/profile.log 2>&1 || { echo "profile failed"; tail -5 $O/profile.log; exit 1; }
mkdir -p $O/summaries && cp gpurun_out/prof_r6v/summaries/* $O/summaries/ && ls $O/summaries
