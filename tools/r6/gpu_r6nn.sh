#!/bin/bash
# cfg4 batches in flight beyond 16 (hardware queues capped at 32)
set -o pipefail
O=gpurun_out/r6nn; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['parity']['ok'])"
}
B="timeout -k 10 200 python -u bench.py --estimator essential --steps 40 --warmup 5 --cpu-seconds 0"
for r in 1 2; do
run p16_$r $B
run p20_$r $B --pipeline 20
run p24_$r $B --pipeline 24
done
