#!/bin/bash
# A/B of branch splitting and stream count on the DPLL bench (run through gpurun):
#   split GPU tests first, then bench lines at configs[2] full size and at the
#   N=8 per-GPU share (32,768 instances), split on/off, 1 and 2 streams.
# Usage: bash tools/split_ab.sh <tag>     -> gpurun_out/<tag>/...
set -o pipefail
TAG=${1:-split_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dpll_gpu.py -k "split or scan_kernel_full or sound_kernels_match or concurrent" \
    -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests_split.log" 2>&1 || { echo "split tests failed"; tail -40 "$OUT/gpu_tests_split.log"; exit 1; }
echo "tests ok"
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
    || { echo "bench $name failed"; tail -20 "$OUT/bench_$name.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$name.json')); print('$name', round(d['value']), 'util', round(d['wave_utilisation'],3), 'kernel_ms', round(d['roofline']['kernel_ms'],1), d.get('branch_split'))"
}
run share_split_s2 --total 32768 --steps 20 --warmup 3
run share_split_s1 --total 32768 --steps 20 --warmup 3 --streams 1
run full_split_s2 --steps 10 --warmup 2
run full_nosplit_s2 --steps 10 --warmup 2 --no-split
grep -h -o '"branch_split": {[^}]*}' "$OUT"/bench_*.json
echo done
