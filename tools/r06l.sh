set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06l; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for e in 0 1; do
  SATMI_DP_INLINE=$e timeout -k 10 100 python bench.py --workload php-dp --steps 40 --warmup 3 --no-cpu-baseline --no-legs > $OUT/b$e.json 2> $OUT/b$e.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b$e.json')); print('inline=$e php-dp', d['value'], d['roofline'])"
done
