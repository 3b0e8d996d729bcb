#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and same-box rate of two library builds on the headline.
# Usage (through gpurun): bash tools/nt_ab.sh <tag> libA.so libB.so
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SATMI_LIB_VARIANT=$lib timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$PWD/$OUT/${lib%.so}_$c" -o p \
      -- python bench.py --steps 2 --warmup 0 --profile-steps --no-legs > "$OUT/${lib%.so}_$c.json" 2> "$OUT/${lib%.so}_$c.err" || { echo "pmc $lib $c failed"; exit 1; }
    f=$(find "$OUT/${lib%.so}_$c" -name '*counter_collection.csv' | head -1)
    echo "$lib $c $(python tools/pmc_sum.py "$f" dpll_fixed_kernel | tail -1)"
    rm -rf "$OUT/${lib%.so}_$c"
  done
done
bash tools/ab.sh "$TAG" 2 - "--steps 8 --warmup 2" "$@"
