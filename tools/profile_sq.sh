#!/bin/bash
# SQ counter passes (two runs of <= 8 SQ counters each) over one bench launch
# of B instances: instruction mix, issue stalls, LDS conflicts of the DPLL kernel.
# Usage: bash tools/profile_sq.sh <tag> [B]     -> gpurun_out/<tag>/sq{1,2}/...
set -eo pipefail
TAG=${1:-sq}
B=${2:-8192}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --output-format csv -d "$ROOT/$OUT/sq1" -o sq1 -- python bench.py --total "$B" --steps 1 --warmup 0 --profile-steps > "$OUT/sq1.json" 2> "$OUT/sq1.err"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$ROOT/$OUT/sq2" -o sq2 -- python bench.py --total "$B" --steps 1 --warmup 0 --profile-steps > "$OUT/sq2.json" 2> "$OUT/sq2.err"
for f in $(find "$OUT/sq1" "$OUT/sq2" -name "*counter_collection.csv"); do python tools/pmc_sum.py "$f"; done > "$OUT/sq_summary.txt"
echo done
