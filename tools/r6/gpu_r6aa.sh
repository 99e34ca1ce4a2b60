#!/bin/bash
# cfg3 exact: polish submission groups and the fused one-workgroup polish
set -o pipefail
O=gpurun_out/r6aa; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['ms_per_step'],4), all(v for k,v in d.get('parity',{}).items() if k!='runs'))"
}
B="timeout -k 10 200 python -u bench.py --sprt-exact --steps 30 --warmup 3 --cpu-seconds 0"
for r in 1 2; do
run g4_$r $B
run g2_$r USAC_POLISH_GROUP=2 $B
run g1_$r USAC_POLISH_GROUP=1 $B
run fused_$r USAC_POLISH_FUSED=1 $B
done
USAC_PROFILE=1 timeout -k 10 200 python -u bench.py --sprt-exact --steps 10 --warmup 2 --cpu-seconds 0 > $O/prof.json 2> $O/prof.err
grep -c "polish" $O/prof.err
