#!/bin/bash
# A/B of DPLL kernel policies on the default bench workload (run through gpurun):
#   optional -m gpu test files first, then one bench line per policy.
# Usage: bash tools/ab_bench.sh <tag> "<test files or ->" <policy>... [-- extra bench args]
set -o pipefail
TAG=$1; TESTS=$2; shift 2
POLICIES=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do POLICIES+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$TESTS" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -v -x --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?
  tail -5 "$OUT/tests.log"
  [ $rc -eq 0 ] || { echo "tests failed ($rc)"; grep -E "Error|assert" "$OUT/tests.log" | head -20; exit 1; }
fi
for p in "${POLICIES[@]}"; do
  timeout -k 10 300 python bench.py --kernel "$p" --no-cpu-baseline "$@" > "$OUT/bench_$p.json" 2> "$OUT/bench_$p.err" \
    || { echo "bench $p failed"; tail -5 "$OUT/bench_$p.err"; exit 1; }
  python - "$OUT/bench_$p.json" "$p" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(f"{sys.argv[2]:8s} value={d['value']:.4g} {d['unit']} kernel_ms={r['kernel_ms']:.1f} "
      f"lds/wave={d['lds_bytes_per_wave']} resident={d['resident_waves']} util={d['wave_utilisation']:.3f}")
EOF
done
