#!/bin/bash
# summarise tools/e5run.sh outputs
tail -2 gpurun_out/t.log
for f in be bf; do [ -f gpurun_out/$f.log ] && tail -1 gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', round(d['value']/1e6,2), 'M/s solve', round(r['solve_kernel_ms'],3), 'score', round(r['kernel_ms'],3), d['parity'])"; done
for p in profe4 proff4; do [ -f gpurun_out/$p/p_kernel_stats.csv ] && python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/$p/p_kernel_stats.csv')))[:8]: print(f\"  {float(r['AverageNs'])/1e3:9.1f} us {r['Calls']:>4} {r['Name'][:60]}\")"; done
