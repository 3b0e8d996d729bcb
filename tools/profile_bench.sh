#!/bin/bash
# Round profile of the benchmark on one MI355X (run through gpurun):
#   bench line, rocprofv3 kernel-trace stats, and HBM traffic of the DPLL kernel
#   from separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md, HBM section).
# Usage: bash tools/profile_bench.sh <tag>      -> gpurun_out/<tag>/...
set -eo pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --full-json "$OUT/bench_full.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o trace \
    -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/fetch" -o fetch \
    -- python bench.py --steps 2 --warmup 0 --profile-steps > "$OUT/fetch_bench.json" 2> "$OUT/fetch.err"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/$OUT/write" -o write \
    -- python bench.py --steps 2 --warmup 0 --profile-steps > "$OUT/write_bench.json" 2> "$OUT/write.err"
# keep the kernel statistics and the counter sums; the per-dispatch rows stay on the box
for d in fetch write; do
  python tools/pmc_sum.py "$(find "$OUT/$d" -name '*counter_collection.csv' | head -1)" > "$OUT/pmc_$d.txt"
  rm -rf "$OUT/$d"
done
find "$OUT/trace" -type f ! -name '*kernel_stats.csv' -delete
echo done
