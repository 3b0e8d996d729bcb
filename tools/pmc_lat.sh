#!/bin/bash
# Latency / back-pressure counters of the headline launch: SQ_ACCUM_PREV_HIRES
# accumulates the one SQ_INST_LEVEL_* counter of its pass (in-flight
# instructions summed over cycles), so ACCUM / INSTS is that kind's average
# latency; the LDS FIFO-full cycles show LDS back-pressure.
# Usage: bash tools/pmc_lat.sh <tag> [bench args]   -> gpurun_out/<tag>/lat.txt
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/lat.txt"
i=0
for grp in "SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES SQ_INSTS_LDS SQ_WAVE_CYCLES" "SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_VMEM SQ_WAVE_CYCLES" \
           "SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_CYCLES_SALU SQ_LDS_ADDR_CONFLICT SQ_BUSY_CU_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$PWD/$OUT/lat$i" -o lat -- python bench.py --steps 1 --warmup 0 \
      --profile-steps --no-legs "$@" > "$OUT/lat$i.json" 2> "$OUT/lat$i.err" || exit 1
  f=$(find "$OUT/lat$i" -name '*counter_collection.csv' | head -1)
  { echo "== pass $i: $grp"; python tools/pmc_sum.py "$f"; } >> "$OUT/lat.txt" || exit 1
  rm -rf "$OUT/lat$i"
done
cat "$OUT/lat.txt"
