#!/bin/bash
# Same-box A/B: libsatmi.so vs libsatmi_v.so (make variant VFLAGS=...), bench lines interleaved.
# Usage: bash tools/ab_variant.sh <tag> <reps> "<bench args>"
set -o pipefail
TAG=$1; REPS=${2:-2}; ARGS=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $REPS); do
  for lib in libsatmi.so libsatmi_v.so; do
    SATMI_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > $OUT/${lib%.so}_$i.json 2>/dev/null || { echo "bench $lib failed"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${lib%.so}_$i.json')); print('$lib', round(d['value']), round(d['roofline']['kernel_ms'],1))"
  done
done
