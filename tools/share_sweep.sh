#!/bin/bash
# N=8-share sweep (run through gpurun from the repo root, library prebuilt):
# full-size headline line, then --total 32768 (one rank's share of 262,144 at N=8)
# under each branch-splitting setting given, `reps` rounds interleaved.
# Usage: bash tools/share_sweep.sh <tag> <reps> "<args>[;<args>...]"
#   -> gpurun_out/<tag>/full_<rep>.json, share_<set>_<rep>.json, one summary line per run
set -o pipefail
TAG=$1; REPS=$2; SETS=$3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
IFS=';' read -r -a ARGSETS <<< "$SETS"
for i in $(seq 1 "$REPS"); do
  f="$OUT/full_$i.json"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 12 --warmup 2 > "$f" 2> "${f%.json}.err" \
      || { echo "full-size bench failed"; tail -5 "${f%.json}.err"; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('full', round(d['value']), round(d['ms_per_step'], 2), d.get('verdict_sha'))"
  for s in "${!ARGSETS[@]}"; do
    f="$OUT/share_${s}_$i.json"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --total 32768 --steps 12 --warmup 2 ${ARGSETS[$s]} \
        > "$f" 2> "${f%.json}.err" || { echo "share [${ARGSETS[$s]}] failed"; tail -5 "${f%.json}.err"; exit 1; }
    python -c "import json; d=json.load(open('$f')); print('share', '[${ARGSETS[$s]}]', round(d['value']), round(d['ms_per_step'], 2), d.get('verdict_sha'))"
  done
done
