#!/bin/bash
# Rehearse the multi-rank bench path on a one-GPU box: torchrun with 2 and 4
# ranks sharing the GPU over gloo (bench.py init_ranks: SATMI_DIST_BACKEND),
# the same --total as a 1-rank run; verdict_sha must agree and n_ranks_seen =
# ranks.  Usage: bash tools/multirank_rehearsal.sh <tag> [total]
set -o pipefail
TAG=$1; TOTAL=${2:-32768}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export SATMI_DIST_BACKEND=gloo
ARGS="--total $TOTAL --steps 3 --warmup 1 --no-cpu-baseline --no-legs"
timeout -k 10 300 python bench.py $ARGS > "$OUT/n1.json" 2> "$OUT/n1.err" || { echo "n1 failed"; tail -5 "$OUT/n1.err"; exit 1; }
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N $ARGS > "$OUT/n$N.json" 2> "$OUT/n$N.err" \
    || { echo "n$N failed"; tail -5 "$OUT/n$N.err"; exit 1; }
done
python - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
rows = []
for n in (1, 2, 4):
    d = json.loads(open(f"{out}/n{n}.json").read().strip().splitlines()[-1])
    rows.append(d)
    print(n, d["n_gpus"], d["verdict_sha"], d["n_ranks_seen"], d["value"], d["config"]["instances_per_gpu"], d["last_step_totals"])
assert len({d["verdict_sha"] for d in rows}) == 1, "verdict hashes differ across rank counts"
assert [d["n_ranks_seen"] for d in rows] == [1, 2, 4]
with open(f"{out}/multirank_rehearsal.jsonl", "w") as fh:
    for d in rows:
        fh.write(json.dumps(d) + "\n")
print("rehearsal ok: same verdict_sha for 1, 2, 4 ranks")
PY
