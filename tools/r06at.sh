# final-tree slices (N = 8, 4, 2; 20 steps / 5 warm-up as slices.json) and the full-size line beside them
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06at; mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 20 --warmup 5 > $OUT/full.json 2> $OUT/full.err || exit 1
python -c "import json; d=json.load(open('$OUT/full.json')); print('full', round(d['value']), round(d['ms_per_step'],2))"
bash tools/slices.sh r06at 8 4 2 || exit 1
