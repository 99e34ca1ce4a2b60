set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
USAC_POLISH_FUSED=${FUSED:-1} USAC_PROFILE=1 timeout -k 10 300 python bench.py --sprt-exact --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/px.json 2> gpurun_out/px.err || { tail -5 gpurun_out/px.err; exit 1; }
grep "polish_fused" gpurun_out/px.err | sed -n "20,26p"
