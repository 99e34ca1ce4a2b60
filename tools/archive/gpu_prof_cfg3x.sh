set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p3x -o run --output-format csv -- python3 $R/bench.py --sprt-exact --steps 30 --warmup 5 --cpu-seconds 0 > $R/gpurun_out/p3x.log 2>&1 || { tail -5 $R/gpurun_out/p3x.log; exit 1; }
find $R/gpurun_out/p3x -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $R/gpurun_out/p3x_stats.csv
