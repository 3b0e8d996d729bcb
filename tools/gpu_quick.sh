#!/bin/bash
# Quick GPU check: selected tests (-k expr) then bench lines (run through gpurun).
# Usage: bash tools/gpu_quick.sh <tag> "<pytest -k expr>" "<bench args>;<bench args>;..."
set -o pipefail
TAG=$1; KEXPR=$2; BENCHES=$3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -k "$KEXPR" -v --timeout 300 --timeout-method thread \
      > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -1 "$OUT/gpu_tests.log"
fi
i=0
IFS=';' read -ra BL <<< "$BENCHES"
for args in "${BL[@]}"; do
  [ -z "$args" ] && continue
  i=$((i+1))
  timeout -k 10 300 python bench.py $args > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" \
    || { echo "bench $i ($args) failed"; tail -20 "$OUT/bench_$i.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); r=d.get('roofline') or {}; print('$args =>', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],2), 'frac', r.get('frac'))"
done
echo done
