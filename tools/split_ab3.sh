#!/bin/bash
# Branch-splitting helper count A/B + the Davis-Putnam tiled filter (run through gpurun).
set -o pipefail
TAG=${1:-split_ab3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_dpll_gpu.py -k "dp or split" \
    -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
echo "tests ok"
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
    || { echo "bench $name failed"; tail -20 "$OUT/bench_$name.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$name.json')); r=d.get('roofline') or {}; print('$name', round(d['value'],1), 'kernel_ms', r.get('kernel_ms'), 'frac', r.get('frac'), (d.get('branch_split') or {}).get('wait_ticks'))"
}
run php_dp --workload php-dp --steps 5 --warmup 2
run php_res --workload php-res --steps 5 --warmup 2
for h in 1 2 8; do
  run share_h$h --total 32768 --steps 20 --warmup 3 --helpers-per-cu $h
done
run full_h1 --steps 10 --warmup 2 --helpers-per-cu 1
echo done
