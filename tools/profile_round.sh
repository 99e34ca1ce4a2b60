#!/bin/bash
# Per-round profiles: per workload a rocprofv3 kernel trace (--stats) of the bench at one batch in
# flight, then separate PMC passes (no PMC + trace mix; <= 8 SQ / 2 GRBM / 4 TCC counters each):
# HBM bytes (FETCH_SIZE, WRITE_SIZE), VALU issue (SQ_ACTIVE_INST_VALU + GRBM_GUI_ACTIVE) and the
# wave-cycle split; cfg2 (h10k) also the scalar data cache (SQC_DCACHE_*) and scalar-memory
# latency (SQ_INST_LEVEL_SMEM / SQ_INSTS_SMEM) passes.  Summaries (tools/summarize_profile.py:
# full-size dispatches only, tagged with the workload shape the bench matches on) go to
# gpurun_out/prof_<tag>/summaries; copy them into profiles/.
#   TAG=r4 WORKLOADS="h10k f10k_sprt f10k_exact e50k" bash tools/profile_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r4}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT/summaries
WORKLOADS=${WORKLOADS:-"h10k f10k_sprt f10k_exact e50k"}
for w in $WORKLOADS; do
  RUNS=""; BATCH=65536; STEPS="--steps 20 --warmup 3"; PSTEPS="--steps 5 --warmup 1"; GRIDS=""
  case $w in
    h10k)       ARGS=""; NPTS=10000 ;;
    h100k)      ARGS="--points 100000"; NPTS=100000 ;;
    e50k)       ARGS="--estimator essential"; NPTS=50000 ;;
    f10k)       ARGS="--estimator fundamental --no-sprt --sampler uniform"; NPTS=10000 ;;
    f10k_sprt)  ARGS="--estimator fundamental"; NPTS=10000; BATCH=262144 ;;   # cfg3: PROSAC + batch SPRT (bench default, B = 262144)
    f10k_exact) ARGS="--sprt-exact"; NPTS=10000; BATCH=1024; STEPS="--steps 20 --warmup 2"; PSTEPS="--steps 5 --warmup 1"; GRIDS=all ;;
    # cfg5 full runs (batch 0 = "whole runs"): every dispatch of warmup + steps + the parity run counts,
    # the summary records the runs so bench.py can put calls per run beside durations
    cfg5)       ARGS="--cfg5"; NPTS=100000; BATCH=0; STEPS="--steps 20 --warmup 2"; PSTEPS="--steps 20 --warmup 2"; GRIDS=all; RUNS=23 ;;
  esac
  D=$OUT/$w; mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$D/trace -o run --output-format csv -- \
      python3 bench.py $STEPS --cpu-seconds 0 --pipeline 1 $ARGS > $D/bench_trace.json 2> $D/trace.err
  rc=$?; echo "== $w trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/trace.err; exit $rc; }
  PASSES=(FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
          "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES")
  if [ $w = h10k ] || [ $w = h100k ] || [ $w = e50k ]; then  # the matrix-core scorers (h16 / e16): MFMA busy, LDS / SALU issue
    PASSES+=("SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE")
  fi
  if [ $w = h10k ]; then
    PASSES+=("SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE"
             "SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES")
  fi
  for ctr in "${PASSES[@]}"; do
    name=$(echo $ctr | tr ' ' '_')
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr -d $PWD/$D/pmc_$name -o run --output-format csv -- \
        python3 bench.py $PSTEPS --cpu-seconds 0 --pipeline 1 $ARGS > $D/bench_pmc_$name.json 2> $D/pmc_$name.err
    rc=$?; echo "== $w pmc $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/pmc_$name.err; exit $rc; }
  done
  python3 tools/summarize_profile.py $D ${TAG}_$w $NPTS $BATCH $OUT/summaries $GRIDS $RUNS > /dev/null || exit 1
  cp $D/trace/run_kernel_stats.csv $OUT/summaries/kernel_stats_${TAG}_$w.csv 2>/dev/null
done
ls -la $OUT/summaries
