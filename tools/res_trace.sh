#!/bin/bash
# Resolution call anatomy (run through gpurun): the -m gpu resolution tests,
# tools/res_time.py, the php-res bench leg, and a kernel trace of 20 calls
# summarised per kernel (gpurun_out/<tag>/).
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_resolution_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 \
    || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 120 python tools/res_time.py > "$OUT/res_time.json" || exit 1
cat "$OUT/res_time.json"
timeout -k 10 120 python bench.py --workload php-res --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['clock_hz'], r['frac'], r['fracs_at_peak_clock'])"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr" -o tr -- python bench.py --workload php-res --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit 1
f=$(find "$OUT/tr" -name '*kernel_stats.csv' | head -1); cp "$f" "$OUT/kernel_stats.csv"
db=$(find "$OUT/tr" -name '*.db' | head -1); [ -n "$db" ] && cp "$db" "$OUT/trace.db"
rm -rf "$OUT/tr"
