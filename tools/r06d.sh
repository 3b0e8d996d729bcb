set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06d; mkdir -p $OUT
for a in 2000 2400 2800; do
  timeout -k 10 100 python tools/fullsolve_probe.py 200 $a 5 5200 64 20 > $OUT/probe_5sat_$a.jsonl 2> $OUT/probe_5sat_$a.err || { tail -5 $OUT/probe_5sat_$a.err; exit 1; }
  tail -1 $OUT/probe_5sat_$a.jsonl | cut -c1-600
done
timeout -k 10 100 python bench.py --no-legs --no-cpu-baseline --steps 5 --warmup 2 > $OUT/full5.json 2>&1 || exit 1
bash tools/slices.sh r06d 8 4 2 > /dev/null || exit 1
python tools/slices_summary.py $OUT/slices.jsonl $OUT/full5.json > $OUT/slices_summary.json || exit 1
python -c "
import json; d=json.load(open('$OUT/slices_summary.json'))
for N,w in d['worlds'].items(): print(N, {k:v for k,v in w.items() if k!='slices'})"
