set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06s; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for w in php-dp rand-dp; do
for e in fixed learned; do
  if [ $e = fixed ]; then export SATMI_DP_FIXED_GRIDS=1; else unset SATMI_DP_FIXED_GRIDS; fi
  SATMI_DP_PHASES=1 timeout -k 10 120 python bench.py --workload $w --steps 40 --warmup 3 --no-cpu-baseline --no-legs > $OUT/$w.$e.json 2> $OUT/$w.$e.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$w.$e.json')); print('$w $e', d['value'], d['ms_per_step'], d['roofline'])"
  tail -1 $OUT/$w.$e.err
done
done
