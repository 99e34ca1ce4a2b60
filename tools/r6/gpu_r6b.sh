#!/bin/bash
# round 6: which VALU classes are corrupted beside MFMA waves; the e16 mismatch detail
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 240 ./tools/mfma_interference 60 > gpurun_out/r6b/interf.log 2>&1; echo "interf rc=$?"
cat gpurun_out/r6b/interf.log
