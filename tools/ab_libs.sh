#!/bin/bash
# Same-box A/B over several in-tree library builds (satmi/<lib>), bench lines interleaved.
# Usage: bash tools/ab_libs.sh <tag> <reps> "<bench args>" lib1.so lib2.so ...
set -o pipefail
TAG=$1; REPS=$2; ARGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $REPS); do
  for lib in "$@"; do
    SATMI_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs $ARGS > $OUT/${lib%.so}_$i.json 2>/dev/null || { echo "bench $lib failed"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${lib%.so}_$i.json')); print('$lib', round(d['value']), round(d['roofline']['kernel_ms'],1))"
  done
done
