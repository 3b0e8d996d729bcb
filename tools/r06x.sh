# N=8 slices with 2 vs 4 streams (default steps 5 / warmup 2, as the driver's default run), and the full size
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06x; mkdir -p $OUT
for ns in 2 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --streams $ns > $OUT/full_s$ns.json 2> $OUT/full_s$ns.err || exit 1
  python -c "import json; d=json.load(open('$OUT/full_s$ns.json')); print('full streams $ns', round(d['value']), round(d['ms_per_step'],2))"
  STEPS=5 WARM=2 EXTRA="--streams $ns" SUFFIX=s$ns bash tools/slices.sh r06x 8 | python -c "
import sys, json
v=[json.loads(l) for l in sys.stdin if l.startswith('{')]
ms=[x['ms_per_step'] for x in v]
print('streams $ns N=8 ms/step', [round(m,2) for m in ms], 'max', round(max(ms),2), 'mean/max', round(sum(ms)/len(ms)/max(ms),3))" || exit 1
done
