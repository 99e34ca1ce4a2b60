#!/bin/bash
set -o pipefail
O=gpurun_out/r6g2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $GRAFT_REPO_ROOT/$O/pmc1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/e16_only.py > $GRAFT_REPO_ROOT/$O/pmc1.log 2>&1; echo "pmc1 rc=$?"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/$O/pmc2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/e16_only.py > $GRAFT_REPO_ROOT/$O/pmc2.log 2>&1; echo "pmc2 rc=$?"
