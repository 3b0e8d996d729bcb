#!/bin/bash
# One rocprofv3 PMC pass per in-tree library build over the same bench launch
# (SQ_LDS_* attribution: `make variant VFLAGS=-DSATMI_DUP_<KIND> VNAME=...`).
# Usage: bash tools/pmc_libs.sh <tag> "<counters>" "<bench args>" lib1.so lib2.so ...
#   -> gpurun_out/<tag>/<lib>/..., summary in gpurun_out/<tag>/summary.txt
set -eo pipefail
TAG=$1; CTRS=$2; ARGS=$3; shift 3
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
  name=${lib%.so}
  SATMI_LIB_VARIANT=$lib timeout -s KILL 150 rocprofv3 --pmc $CTRS --output-format csv -d "$ROOT/$OUT/$name" -o pmc \
      -- python bench.py --steps 1 --warmup 0 --profile-steps $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
  echo "== $lib" >> "$OUT/summary.txt"
  python tools/pmc_sum.py "$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)" >> "$OUT/summary.txt" && rm -rf "$OUT/$name"
  echo "$lib ok"
done
cat "$OUT/summary.txt"
