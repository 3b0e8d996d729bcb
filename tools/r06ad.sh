set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06ad; mkdir -p $OUT
timeout -k 10 300 python bench.py --workload uf250 --node-limit 0 --total 1024 --split-always --helpers-per-cu 16 --steps 2 --warmup 0 --no-cpu-baseline --no-legs > $OUT/uf250s.json 2> $OUT/uf250s.err || exit 1
python -c "import json; d=json.load(open('$OUT/uf250s.json')); print('uf250 solved', d['value'], d['unit'], d.get('wave_utilisation'), d['verdict_sha'])"
for h in 2 4; do
STEPS=5 WARM=2 EXTRA="--helpers-per-cu $h" SUFFIX=h$h bash tools/slices.sh r06ad 8 | python -c "
import sys, json
v=[json.loads(l) for l in sys.stdin if l.startswith('{')]
ms=[x['ms_per_step'] for x in v]
print('helpers $h N=8 ms/step', [round(m,2) for m in ms], 'max', round(max(ms),2), 'mean/max', round(sum(ms)/len(ms)/max(ms),3))" || exit 1
done
