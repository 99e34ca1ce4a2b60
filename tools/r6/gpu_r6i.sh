#!/bin/bash
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_e5_rpoly.py tests/test_gpu_essential.py tests/test_gpu_e16.py tests/test_gpu_baseline_sizes.py tests/test_gpu_sharded_run.py tests/test_gpu_mfma_concurrency.py > $O/tests.log 2>&1; echo "tests rc=$?"; tail -4 $O/tests.log
timeout -k 10 100 python -u tools/e_phase.py > $O/phase.log 2>&1; echo "phase rc=$?"; cat $O/phase.log
for P in 3 6; do GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 0 --pipeline $P > $O/bench_p$P.json 2> $O/bench_p$P.err; echo "pipeline $P rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_p$P.json'));print(d['value']/1e6, d['ms_per_step'])"; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o e --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/e_phase.py > /dev/null 2>&1; echo "prof rc=$?"
