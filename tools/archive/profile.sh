#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then separate PMC passes (no PMC+trace mix).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
STEPS=${STEPS:-20}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps $STEPS --warmup 3 --cpu-seconds 0 ${BENCH_ARGS:-} > $OUT/bench_trace.json 2> $OUT/trace.err
rc=$?; echo "== trace rc=$rc"; cat $OUT/bench_trace.json; tail -5 $OUT/trace.err
[ $rc -eq 0 ] || exit $rc
for ctr in ${PMC:-FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"}; do
  name=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/pmc_$name -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} > $OUT/bench_pmc_$name.json 2> $OUT/pmc_$name.err
  rc=$?; echo "== pmc $ctr rc=$rc"; tail -3 $OUT/pmc_$name.err
  [ $rc -eq 0 ] || exit $rc
done
find $OUT -name "*.csv" | head -50
