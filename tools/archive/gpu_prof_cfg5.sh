set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p5 -o run --output-format csv -- python3 $R/bench.py --cfg5 --steps 10 --warmup 3 --cpu-seconds 0 > $R/gpurun_out/p5.log 2>&1 || { tail -5 $R/gpurun_out/p5.log; exit 1; }
cp $R/gpurun_out/p5/*kernel_stats.csv $R/gpurun_out/p5_stats.csv 2>/dev/null || find $R/gpurun_out/p5 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/p5_stats.csv \;
cd $R && USAC_PROFILE=1 timeout -k 10 300 python bench.py --cfg5 --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/p5b.json 2> gpurun_out/p5b.err
grep "usac_ransac_run ms" gpurun_out/p5b.err | tail -3
