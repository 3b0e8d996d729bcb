set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06u}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for w in php-dp rand-dp; do
  timeout -k 10 120 python bench.py --workload $w --steps 40 --warmup 3 --no-cpu-baseline --no-legs > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/tr" -o t -- python tools/dp_trace_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
f=$(find "$OUT/tr" -name '*kernel_trace.csv' | head -1)
cp "$f" $OUT/kernel_trace.csv
rm -rf $OUT/tr
