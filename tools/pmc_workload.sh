#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a bench workload,
# summed per kernel substring: issue mix, L2 hits/misses, HBM FETCH / WRITE.
# Usage: [PMC_GROUPS="sq1 sq2 tcc fetch write"] bash tools/pmc_workload.sh <tag> <workload> "<kernel substrings>" [bench args]
#   -> gpurun_out/<tag>/pmc_<workload>.txt (+ p<i>.json: the bench line of each pass)
set -o pipefail
TAG=$1; WL=$2; KS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
SUM="$OUT/pmc_$WL.txt"
: > "$SUM"
i=0
PASSES=${PMC_GROUPS:-"sq1 sq2 tcc fetch write"}
declare -A G=(
  [sq1]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  [sq2]="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  [tcc]="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum"
  [fetch]="FETCH_SIZE" [write]="WRITE_SIZE")
for gname in $PASSES; do
  grp=${G[$gname]}
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/p$i" -o p$i \
    -- python bench.py --workload "$WL" --no-cpu-baseline "$@" > "$OUT/p$i.json" 2> "$OUT/p$i.err" \
    || { echo "pass $i ($grp) failed"; tail -3 "$OUT/p$i.err"; exit 1; }
  f=$(find "$OUT/p$i" -name '*counter_collection.csv' | head -1)
  for k in $KS; do echo "== pass $i kernel $k"; python tools/pmc_sum.py "$f" "$k"; done >> "$SUM"
  rm -rf "$OUT/p$i"
done
cat "$SUM"
