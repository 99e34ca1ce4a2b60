#!/bin/bash
# pipeline depth sweep on the default (cfg2) bench
for P in 1 2 3 4 6; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --pipeline $P > gpurun_out/ps.log 2>&1 || { tail -3 gpurun_out/ps.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ps.log').read().strip().splitlines()[-1]); r=d['roofline']; print('P=$P %8.2f M/s ms/step %.4f score %.4f solve %.4f' % (d['value']/1e6, d['ms_per_step'], r['kernel_ms'], r['solve_kernel_ms']))"
done
