#!/bin/bash
# End-of-round evidence: GPU tests, smoke, every bench line, rocprofv3 traces of each mode,
# PMC passes (HBM bytes, VALU) of the headline kernel.  Outputs under gpurun_out/round/.
set -u
OUT=${OUT:-gpurun_out/round}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 900 bash tools/bench_all.sh > $OUT/bench_all.txt 2>&1 || { cat $OUT/bench_all.txt; exit 1; }
cat $OUT/bench_all.txt
timeout -k 10 300 python bench.py --cfg5 > $OUT/cfg5.json 2>$OUT/cfg5.err || { tail -5 $OUT/cfg5.err; exit 1; }
cat $OUT/cfg5.json
USAC_PROFILE=1 timeout -k 10 300 python tools/feature_bench.py > $OUT/features.json 2> $OUT/features.err || { tail -5 $OUT/features.err; exit 1; }
cat $OUT/features.json
timeout -k 10 200 python tools/score_vs_inliers.py > $OUT/score_vs_inliers.txt 2>&1 || exit 1
cat $OUT/score_vs_inliers.txt
if [ -x tools/ubench/valu_rate ]; then timeout -k 10 60 ./tools/ubench/valu_rate > $OUT/valu_rate.txt 2>&1 || exit 1; cat $OUT/valu_rate.txt; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/trace_cfg5 -o run --output-format csv -- \
    python3 bench.py --cfg5 --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/trace_cfg5.json 2> $OUT/trace_cfg5.err || { echo "trace cfg5 failed"; exit 1; }
for mode in "h:" "f:--estimator fundamental" "e:--estimator essential"; do
  tag=${mode%%:*}; args=${mode#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/trace_$tag -o run --output-format csv -- \
      python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --pipeline 1 $args > $OUT/trace_$tag.json 2> $OUT/trace_$tag.err || { echo "trace $tag failed"; exit 1; }
done
for ctr in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  name=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $PWD/$OUT/pmc_$name -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --pipeline 1 > $OUT/pmc_$name.json 2> $OUT/pmc_$name.err || { echo "pmc $ctr failed"; exit 1; }
done
echo done
