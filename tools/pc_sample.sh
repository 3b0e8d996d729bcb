#!/bin/bash
# PC sampling (rocprofv3 beta, host trap) over a short bench run (run through gpurun).
set -o pipefail
TAG=${1:-pcs}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
rocprofv3 -L > "$OUT/list_avail.txt" 2>&1 || true
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 1 --output-format csv -d "$ROOT/$OUT/pcs" -o pcs \
    -- python bench.py --total 32768 --steps 2 --warmup 0 --profile-steps > "$OUT/bench.json" 2> "$OUT/pcs.err"
echo "rc=$?"
ls -la "$OUT/pcs" 2>/dev/null | head; find "$OUT/pcs" -name "*.csv" | head
