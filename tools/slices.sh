#!/bin/bash
# The 8-GPU (and 4-GPU) imbalance bound on one GPU:
# every rank's shard of the configs[2] batch, run alone on this GPU with
# bench.py --emulate-world N --emulate-rank r, one line per slice.
#   [EXTRA="--split-always ..."] [SUFFIX=x] bash tools/slices.sh <tag> [worlds...]     (default: 8 4)
# -> gpurun_out/<tag>/slices.jsonl; summarise with tools/slices_summary.py
set -o pipefail
TAG=${1:-slices}
shift || true
WORLDS=${*:-8 4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/slices$SUFFIX.jsonl"
for N in $WORLDS; do
  for r in $(seq 0 $((N - 1))); do
    timeout -k 10 300 python bench.py --emulate-world "$N" --emulate-rank "$r" --no-cpu-baseline --no-legs \
      --steps ${STEPS:-20} --warmup ${WARM:-5} $EXTRA > "$OUT/slice${SUFFIX}_${N}_${r}.json" 2> "$OUT/slice${SUFFIX}_${N}_${r}.err" \
      || { echo "slice $N/$r failed"; tail -5 "$OUT/slice${SUFFIX}_${N}_${r}.err"; exit 1; }
    python -c "
import json; d = json.load(open('$OUT/slice${SUFFIX}_${N}_${r}.json'))
print(json.dumps({'world': $N, 'rank': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'shard': d['config']['emulated_shard'], 'verdict_sha': d['verdict_sha'],
                  'sat': d['last_step_totals']['sat'], 'kernel_ms': d['roofline']['kernel_ms'],
                  'split': (d.get('branch_split') or {}).get('donations'), 'extra': '$EXTRA'}))" >> "$OUT/slices$SUFFIX.jsonl"
    tail -1 "$OUT/slices$SUFFIX.jsonl"
  done
done
