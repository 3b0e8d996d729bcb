set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06t; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/tr" -o t -- python tools/dp_trace_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
f=$(find "$OUT/tr" -name '*kernel_trace.csv' | head -1)
cp "$f" $OUT/kernel_trace.csv
rm -rf $OUT/tr
wc -l $OUT/kernel_trace.csv
