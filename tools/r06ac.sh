set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06ac; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_dpll_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py --workload uf250 --total 1024 --split-always --helpers-per-cu 16 --steps 2 --warmup 0 --no-cpu-baseline --no-legs > $OUT/uf250s.json 2> $OUT/uf250s.err || exit 1
python -c "import json; d=json.load(open('$OUT/uf250s.json')); print('uf250 solved', d['value'], d.get('wave_utilisation'), d['verdict_sha'])"
STEPS=5 WARM=2 bash tools/slices.sh r06ac 8 | python -c "
import sys, json
v=[json.loads(l) for l in sys.stdin if l.startswith('{')]
ms=[x['ms_per_step'] for x in v]
print('N=8 ms/step', [round(m,2) for m in ms], 'max', round(max(ms),2), 'mean/max', round(sum(ms)/len(ms)/max(ms),3))"
