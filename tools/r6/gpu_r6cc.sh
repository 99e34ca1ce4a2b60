#!/bin/bash
# packed-fp32-ops off in the backend with the vectorisers on ("feat") vs the vectorisers off ("cur"):
# the race reproducer, the concurrency tests, then cfg3 / cfg4 / cfg2 / cfg5 same-box lines
set -o pipefail
O=gpurun_out/r6cc; mkdir -p $O
timeout -k 10 300 ./tools/h16_race > $O/race.log 2>&1; echo "race rc=$?"; grep "^mode" $O/race.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_mfma_concurrency.py tests/test_gpu_loop.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,3), round(d['ms_per_step'],4), all(v for k,v in d.get('parity',{}).items() if k not in ('runs',)) if 'ok' not in d.get('parity',{}) else d['parity']['ok'])"
}
for r in 1 2; do for v in cur feat; do
L=RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so
run f_${v}_$r $L timeout -k 10 200 python -u bench.py --estimator fundamental --steps 20 --warmup 5 --cpu-seconds 0
run e_${v}_$r $L timeout -k 10 200 python -u bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0
run h_${v}_$r $L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0
run c5_${v}_$r $L timeout -k 10 300 python -u bench.py --cfg5 --steps 20 --warmup 2 --cpu-seconds 0
run c3x_${v}_$r $L timeout -k 10 200 python -u bench.py --sprt-exact --steps 20 --warmup 3 --cpu-seconds 0
done; done
