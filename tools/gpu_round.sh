#!/bin/bash
# One GPU verification pass (run through gpurun from the repo root, library prebuilt):
#   -m gpu suite (verbose log kept), smoke(), bench line, kernel trace + HBM PMC
#   passes (tools/profile_bench.sh), SQ/LDS PMC passes (tools/profile_sq.sh),
#   HBM PMC passes of the resolution leg (php-res, 2 steps: FETCH_SIZE / WRITE_SIZE
#   summed per kernel, every dispatch of both steps).
# Usage: bash tools/gpu_round.sh <tag> [steps...]   steps: tests smoke prof sq res (default all)
set -o pipefail
TAG=${1:-round}
shift || true
STEPS=${*:-tests smoke prof sq res}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
             > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; } ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
             || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; } ;;
    prof)  bash tools/profile_bench.sh "$TAG" || { echo "profile_bench failed"; exit 1; } ;;
    sq)    bash tools/profile_sq.sh "$TAG" || { echo "profile_sq failed"; exit 1; } ;;
    res)   for c in FETCH_SIZE WRITE_SIZE; do
             timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$PWD/$OUT/res_$c" -o res \
               -- python bench.py --workload php-res --steps 2 --warmup 0 --profile-steps --no-cpu-baseline \
               > "$OUT/res_$c.json" 2> "$OUT/res_$c.err" || { echo "res pass $c failed"; exit 1; }
             f=$(find "$OUT/res_$c" -name '*counter_collection.csv' | head -1)
             for k in ht_cand res_pairs ""; do echo "== ${k:-all kernels}"; python tools/pmc_sum.py "$f" $k; done > "$OUT/res_pmc_$c.txt"
             rm -rf "$OUT/res_$c"
           done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
tail -3 "$OUT/gpu_tests.log" 2>/dev/null
cat "$OUT/bench.json" 2>/dev/null || true
