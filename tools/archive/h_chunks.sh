#!/bin/bash
for C in 8 16; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --chunks $C > gpurun_out/hc.log 2>&1 || { tail -3 gpurun_out/hc.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/hc.log').read().strip().splitlines()[-1]); r=d['roofline']; print('C=$C %8.2f M/s ms/step %.4f score %.4f solve %.4f parity %s' % (d['value']/1e6, d['ms_per_step'], r['kernel_ms'], r['solve_kernel_ms'], d['parity']['scores_bit_equal']))"
done
