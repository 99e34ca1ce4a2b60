#!/bin/bash
# PMC pass over cfg5 runs (wave-cycle split and VALU issue per LO kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $PWD/gpurun_out/pmc5 -o run --output-format csv -- python3 tools/cfg5_split.py 3 > /dev/null 2> gpurun_out/pmc5.err || exit $?
