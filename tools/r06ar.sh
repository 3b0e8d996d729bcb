set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06ar; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --workload cdcl --steps 3 --warmup 1 --threads 4 --no-cpu-baseline --no-legs > $OUT/c4_$i.json 2> $OUT/c4_$i.err || exit 1
  python -c "import json; d=json.load(open('$OUT/c4_$i.json')); print('cdcl 4 threads', round(d['value']), round(d['ms_per_step'],2))"
  timeout -k 10 120 python bench.py --workload cdcl --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $OUT/c1_$i.json 2> $OUT/c1_$i.err || exit 1
  python -c "import json; d=json.load(open('$OUT/c1_$i.json')); print('cdcl 1 thread', round(d['value']), round(d['ms_per_step'],2))"
done
