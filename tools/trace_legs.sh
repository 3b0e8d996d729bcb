#!/bin/bash
# rocprofv3 kernel-trace statistics of each non-headline workload (one run each, no CPU baseline),
# kept as gpurun_out/<tag>/<workload>_kernel_stats.csv.  Usage (through gpurun): bash tools/trace_legs.sh <tag>
set -o pipefail
TAG=${1:-legtrace}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in "php-res --steps 20 --warmup 2" "php-dp --steps 20 --warmup 2" "rand-res --steps 3 --warmup 1" \
          "rand-dp --steps 3 --warmup 1" "uf250 --steps 2 --warmup 1" "5sat-n200 --steps 2 --warmup 1" \
          "cdcl --steps 3 --warmup 1"; do
  name=${wl%% *}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/$name" -o t \
      -- python bench.py --workload $wl --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; exit 1; }
  f=$(find "$OUT/$name" -name '*kernel_stats.csv' | head -1)
  cp "$f" "$OUT/${name}_kernel_stats.csv"
  rm -rf "$OUT/$name"
  echo "$name ok"
done
