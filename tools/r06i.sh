set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_driver_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for w in php-dp rand-dp; do
  timeout -k 10 200 python bench.py --workload $w --steps 40 --warmup 3 --no-cpu-baseline --no-legs > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); r=d['roofline'] or {}; print('$w', d['value'], d['ms_per_step'], r.get('launches_per_solve'), r.get('device_ms_per_solve'), r.get('frac'))"
done
timeout -k 10 200 python bench.py --workload php-dp --threads 8 --steps 10 --warmup 2 --no-cpu-baseline --no-legs > $OUT/php8.json 2> $OUT/php8.err || exit 1
python -c "import json; d=json.load(open('$OUT/php8.json')); print('php-dp 8 threads', d['value'])"
