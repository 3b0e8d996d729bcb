#!/bin/bash
# SQ counter passes over one bench launch of B instances (default: the full
# configs[2] step, 262,144 x n=100): instruction mix, issue stalls, LDS-array
# cycles and bank conflicts of the DPLL kernel, plus GRBM_GUI_ACTIVE (chip
# clock x XCDs) for the issue / LDS fractions (tools/sq_roofline.py).
# Usage: bash tools/profile_sq.sh <tag> [B] [extra bench args]   -> gpurun_out/<tag>/sq{1,2}/...
set -eo pipefail
TAG=${1:-sq}
B=${2:-262144}
shift $(( $# < 2 ? $# : 2 ))
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d "$ROOT/$OUT/sq1" -o sq1 -- python bench.py --total "$B" --steps 1 --warmup 0 --profile-steps "$@" > "$OUT/sq1.json" 2> "$OUT/sq1.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    --output-format csv -d "$ROOT/$OUT/sq2" -o sq2 -- python bench.py --total "$B" --steps 1 --warmup 0 --profile-steps "$@" > "$OUT/sq2.json" 2> "$OUT/sq2.err"
for f in $(find "$OUT/sq1" "$OUT/sq2" -name "*counter_collection.csv"); do python tools/pmc_sum.py "$f"; done > "$OUT/sq_summary.txt"
rm -rf "$OUT/sq1" "$OUT/sq2"   # per-dispatch rows: only the summary comes back (gpurun_out <= 64 MiB)
echo done
