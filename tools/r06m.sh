set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --full-json $OUT/bench_full.json > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
wc -c $OUT/bench.json
python -c "
import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['wall_s'], d['cpu_baseline'])
for k,v in d['configs'].items(): print(k, v['value'], v['unit'], v.get('wave_utilisation'), v['cpu_baseline'])"
