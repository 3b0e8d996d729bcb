set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ag}; mkdir -p $OUT
for h in ${HS:-1 2 4}; do
  timeout -k 10 300 python bench.py --workload 5sat-n200-a12 --total 16384 --split-always --helpers-per-cu $h --steps ${ST:-2} --warmup 0 --no-cpu-baseline --no-legs > $OUT/h$h.json 2> $OUT/h$h.err || exit 1
  python -c "import json; d=json.load(open('$OUT/h$h.json')); print('5sat solved helpers $h', round(d['value'],1), d['unit'], round(d['ms_per_step'],1), d.get('wave_utilisation'), d['verdict_sha'])"
done
