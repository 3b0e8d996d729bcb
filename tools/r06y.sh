# cost of the SPLIT kernel form: full size split-always vs default (unsplit), and the N=8 slice 0 split vs unsplit
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06y}; mkdir -p $OUT
for v in "full_def:" "full_split:--split-always" "s8_def:--emulate-world 8 --emulate-rank 0" "s8_nosplit:--emulate-world 8 --emulate-rank 0 --no-split" "full_def2:" "full_split2:--split-always"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 8 --warmup 2 $a > $OUT/$n.json 2> $OUT/$n.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],2), d['roofline']['kernel'], d.get('wave_utilisation'))"
done
