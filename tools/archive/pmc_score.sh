#!/bin/bash
# PMC passes over the default bench for one library build (score-kernel counters):
# pmc_score.sh <lib.so> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIB=$1; shift
export RANSAC_AMD_LIB=$PWD/$LIB
name=$(basename $LIB .so)
OUT=gpurun_out/pmc_$name; mkdir -p $OUT
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 5 -s KILL 90 rocprofv3 --pmc $ctr -d $PWD/$OUT/p$i -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --pipeline 1 "$@" > $OUT/b$i.json 2> $OUT/p$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "pmc pass $i rc=$rc"; tail -3 $OUT/p$i.err; exit $rc; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "score" not in k:
            continue
        acc[k[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %14.1f" % (c, sum(v) / max(1, len(v))))
PY
