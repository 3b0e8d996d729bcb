#!/bin/bash
# configs[4] solved to the end (no node limit): one step per run, branch
# splitting always, over instance counts and helpers per CU.
# Usage: bash tools/fullsolve_sweep.sh <tag> <workload> "<total>:<helpers>[ ...]" [extra bench args]
set -o pipefail
TAG=$1; WL=$2; RUNS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $RUNS; do
  T=${r%%:*}; H=${r##*:}
  f="$OUT/${WL}_${T}_h${H}.json"
  timeout -k 10 240 python bench.py --workload "$WL" --node-limit 0 --total "$T" --split-always --helpers-per-cu "$H" \
      --steps 1 --warmup 0 --no-cpu-baseline --no-legs "$@" > "$f" 2> "${f%.json}.err" \
      || { echo "run $r failed"; tail -5 "${f%.json}.err"; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('$WL', '$r', round(d['value'], 2), round(d['ms_per_step']), 'util', round(d['wave_utilisation'], 3), d['verdict_sha'], d['sat_fraction'])"
done
