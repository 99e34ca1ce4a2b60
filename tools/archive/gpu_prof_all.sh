set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=r5g WORKLOADS="h10k f10k_sprt f10k_exact e50k" bash tools/profile_round.sh > gpurun_out/prof_all.log 2>&1 || { tail -20 gpurun_out/prof_all.log; exit 1; }
tail -8 gpurun_out/prof_all.log
