set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06c; mkdir -p $OUT
for a in 3000 3400 3800; do
  timeout -k 10 100 python tools/fullsolve_probe.py 200 $a 5 5200 64 30 > $OUT/probe_5sat_$a.jsonl 2> $OUT/probe_5sat_$a.err || { tail -5 $OUT/probe_5sat_$a.err; exit 1; }
  tail -1 $OUT/probe_5sat_$a.jsonl | cut -c1-400
done
SUFFIX=_un bash tools/slices.sh r06c 8 4 2 > /dev/null || exit 1
EXTRA="--split-always" SUFFIX=_sa bash tools/slices.sh r06c 8 4 2 > /dev/null || exit 1
EXTRA="--split-always --split-warmup 64" SUFFIX=_saw64 bash tools/slices.sh r06c 8 4 > /dev/null || exit 1
for s in _un _sa _saw64; do python - $s <<'PY'
import json, sys
rows = [json.loads(x) for x in open(f"gpurun_out/r06c/slices{sys.argv[1]}.jsonl")]
for N in (8, 4, 2):
    ms = [r["ms_per_step"] for r in rows if r["world"] == N]
    if ms: print(sys.argv[1], N, "mean/max %.3f" % (sum(ms) / len(ms) / max(ms)), "max %.2f" % max(ms), "mean rate %.0f" % (sum(r["value"] for r in rows if r["world"] == N) / len(ms)))
PY
done
