set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06f; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for h in 1 10; do
  timeout -k 10 200 python bench.py --workload 5sat-n200-a12 --split-always --helpers-per-cu $h --steps 2 --warmup 1 --no-cpu-baseline --no-legs > $OUT/a12_h$h.json 2> $OUT/a12_h$h.err || { tail -5 $OUT/a12_h$h.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/a12_h$h.json')); print('a12 h$h', d['value'], d['ms_per_step'], d['wave_utilisation'], d['verdict_sha'], d['branch_split'])"
done
for h in 10 4; do
  timeout -k 10 300 python bench.py --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu $h --steps 2 --warmup 0 --no-cpu-baseline --no-legs > $OUT/uf_h$h.json 2> $OUT/uf_h$h.err || { tail -5 $OUT/uf_h$h.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/uf_h$h.json')); print('uf250 h$h', d['value'], d['ms_per_step'], d['wave_utilisation'], d['verdict_sha'], d['branch_split'])"
done
STEPS=20 WARM=5 bash tools/slices.sh r06f 8 > /dev/null || exit 1
timeout -k 10 100 python bench.py --no-legs --no-cpu-baseline --steps 20 --warmup 5 > $OUT/full.json 2>&1 || exit 1
python tools/slices_summary.py $OUT/slices.jsonl $OUT/full.json > $OUT/slices_summary.json && python -c "
import json; d=json.load(open('$OUT/slices_summary.json')); print(d['full_size']); [print(N, {k:v for k,v in w.items() if k!='slices'}) for N,w in d['worlds'].items()]"
