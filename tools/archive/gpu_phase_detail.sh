set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
USAC_PROFILE=1 timeout -k 10 300 python bench.py --sprt-exact --steps 60 --warmup 5 --cpu-seconds 0 > gpurun_out/px.json 2> gpurun_out/px.err || { tail -5 gpurun_out/px.err; exit 1; }
python3 - <<'PY'
import re, numpy as np
rows=[l for l in open('gpurun_out/px.err') if l.startswith('usac_ransac_run ms')]
w=np.array([[float(x) for x in re.findall(r'sprt walks ([0-9.]+), draws ([0-9.]+)', l)[0]] for l in rows[5:65]])
ph=np.array([list(map(float, re.findall(r"(?:setup|draw|device|sums|replay|lo|polish) ([0-9.]+)", l))) for l in rows[5:65]])
print('phases', ph.mean(0).round(3), 'walks, draws', w.mean(0).round(3))
PY
python3 - <<'PY'
import re
rows=[l for l in open('gpurun_out/px.err') if l.startswith('usac_ransac_run ms')]
for l in rows[:70]:
    v=re.findall(r"(setup|draw|device|polish) ([0-9.]+)", l); it=re.findall(r"iters (\d+) batches (\d+)", l)
    print(' '.join(b for a,b in v), it)
PY
