#!/bin/bash
# cfg4: batches in flight beyond 8 (N = 1) and hardware queues
set -o pipefail
O=gpurun_out/r6u; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
}
B="timeout -k 10 200 python -u bench.py --estimator essential --steps 30 --warmup 5 --cpu-seconds 0"
run p8 $B --pipeline 8
run p12 $B --pipeline 12
run p16 $B --pipeline 16
run p12_q24 GPU_MAX_HW_QUEUES=24 $B --pipeline 12
run p16_q32 GPU_MAX_HW_QUEUES=32 $B --pipeline 16
run p8b $B --pipeline 8
