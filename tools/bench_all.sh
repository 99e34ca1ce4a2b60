#!/bin/bash
# All bench modes of the round (1 GPU): one JSON line each under gpurun_out/bench_all/
set -u
OUT=gpurun_out/bench_all
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $OUT/$name.log; exit 1; }
  tail -1 $OUT/$name.log > $OUT/$name.json
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('%-16s %8.2f M hyp/s  ms/step %.3f  score %.3f  solve %.3f  parity %s' % ('$name', d['value']/1e6, d['ms_per_step'], r['kernel_ms'], r['solve_kernel_ms'], d.get('parity',{}).get('inlier_counts_equal')))"
}
run h_cfg2
run h_sprt_b262k --sprt --batch 262144 --cpu-seconds 0
run f_cfg3 --estimator fundamental
run f_full_uniform --estimator fundamental --no-sprt --sampler uniform --cpu-seconds 0
run f_full_b262k --estimator fundamental --no-sprt --sampler uniform --batch 262144 --cpu-seconds 0
run f_cfg3_b262k --estimator fundamental --batch 262144 --cpu-seconds 0
run e_cfg4 --estimator essential
run e_b262k --estimator essential --batch 262144 --cpu-seconds 0
run e_sprt --estimator essential --sprt --cpu-seconds 0
run n_napsac --sampler napsac --cpu-seconds 0
