#!/bin/bash
# cfg4: e16 point chunks (USAC_E16_CHUNKS; default ~30 for 26 k listed models) and batches in flight
set -o pipefail
O=gpurun_out/r6gg; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
}
B="timeout -k 10 200 python -u bench.py --estimator essential --steps 30 --warmup 5 --cpu-seconds 0"
for r in 1 2; do
run def_$r $B
run c16_$r USAC_E16_CHUNKS=16 $B
run c48_$r USAC_E16_CHUNKS=48 $B
run c64_$r USAC_E16_CHUNKS=64 $B
run p16_$r $B --pipeline 16
done
