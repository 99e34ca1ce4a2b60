#!/bin/bash
# hardware queues per process vs batches in flight: cfg4 and cfg2 lines
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
}
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0"
run e_q8   GPU_MAX_HW_QUEUES=8  USAC_E16=1 $B --estimator essential
run e_q16  GPU_MAX_HW_QUEUES=16 USAC_E16=1 $B --estimator essential
run e_q32  GPU_MAX_HW_QUEUES=32 USAC_E16=1 $B --estimator essential
run e_q16_p6 GPU_MAX_HW_QUEUES=16 USAC_E16=1 $B --estimator essential --pipeline 6
run e_q16_f2 GPU_MAX_HW_QUEUES=16 USAC_E16=0 $B --estimator essential
run h_q4   GPU_MAX_HW_QUEUES=4  $B
run h_q8   GPU_MAX_HW_QUEUES=8  $B
run h_q16  GPU_MAX_HW_QUEUES=16 $B
run h_q16_p4 GPU_MAX_HW_QUEUES=16 $B --pipeline 4
run f_q4   GPU_MAX_HW_QUEUES=4  $B --estimator fundamental
run f_q16  GPU_MAX_HW_QUEUES=16 $B --estimator fundamental
