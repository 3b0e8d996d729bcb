#!/bin/bash
# Same-box A/B (run through gpurun from the repo root, libraries prebuilt in-tree):
# optional -m gpu tests first, then bench lines interleaved over library builds
# (satmi/<lib>: `make variant VFLAGS=... VNAME=...`, or an older tree's build)
# and bench argument sets, `reps` rounds.
# Usage: bash tools/ab.sh <tag> <reps> "<pytest -k expr | ->" "<bench args>[;<bench args>...]" lib.so...
#   -> gpurun_out/<tag>/<lib>_<set>_<rep>.json, one summary line per run on stdout
set -o pipefail
TAG=$1; REPS=$2; KEXPR=$3; SETS=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$KEXPR" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" \
      > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
IFS=';' read -r -a ARGSETS <<< "$SETS"
for i in $(seq 1 "$REPS"); do
  for s in "${!ARGSETS[@]}"; do
    for lib in "$@"; do
      f="$OUT/${lib%.so}_${s}_$i.json"
      SATMI_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs ${ARGSETS[$s]} \
          > "$f" 2> "${f%.json}.err" || { echo "bench $lib [${ARGSETS[$s]}] failed"; tail -5 "${f%.json}.err"; exit 1; }
      python -c "import json; d=json.load(open('$f')); print('$lib', '[${ARGSETS[$s]}]', round(d['value']), round(d['ms_per_step'], 2))"
    done
  done
done
