#!/bin/bash
# cfg5 / cfg3-exact cost of the no-packed-fp32 rule (diagnostic packed build) and of h16 in the loop
set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,4), round(d['ms_per_step'],4), all(v for k,v in d.get('parity',{}).items() if k!='runs'))"
}
B5="timeout -k 10 300 python -u bench.py --cfg5 --steps 20 --warmup 2 --cpu-seconds 0"
B3="timeout -k 10 200 python -u bench.py --sprt-exact --steps 20 --warmup 3 --cpu-seconds 0"
for r in 1 2; do
run c5_cur_$r RANSAC_AMD_LIB=ransac_amd/var_libs/lib_cur.so $B5
run c5_pk_$r RANSAC_AMD_LIB=ransac_amd/var_libs/lib_packed.so $B5
run c5_h16_$r RANSAC_AMD_LIB=ransac_amd/var_libs/lib_cur.so USAC_LOOP_H16=1 $B5
done
run c3_cur RANSAC_AMD_LIB=ransac_amd/var_libs/lib_cur.so $B3
run c3_pk RANSAC_AMD_LIB=ransac_amd/var_libs/lib_packed.so $B3
