#!/bin/bash
# Quick GPU iteration (run through gpurun from the repo root, library prebuilt):
#   bash tools/gpu_quick.sh <tag> "<pytest files>" "<bench workloads>" [prof]
# -> gpurun_out/<tag>/: tests.log, b_<w>.json, and with `prof` a rocprofv3
#    kernel trace per workload summarised by tools/prof_summary.py.
set -o pipefail
TAG=$1; TESTS=$2; WLS=$3; PROF=$4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -4 "$OUT/tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$OUT/tests.log" | head -20; exit 1; }
fi
for w in $WLS; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/b_$w.json" 2> "$OUT/b_$w.err" \
    || { echo "bench $w failed"; tail -5 "$OUT/b_$w.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/b_$w.json')); print('$w', d['value'], d['unit'], d['ms_per_step'], 'ms/step')"
  if [ "$PROF" = prof ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_$w" -o k -- python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> "$OUT/prof_$w.err" \
      || { echo "prof $w failed"; exit 1; }
  fi
done
exit 0
