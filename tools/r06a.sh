set -o pipefail
OUT=gpurun_out/r06a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --full-json $OUT/bench_full.json > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
wc -c $OUT/bench.json
timeout -k 10 100 python bench.py --no-legs --no-cpu-baseline --steps 5 --warmup 2 > $OUT/full5.json 2>&1 || exit 1
bash tools/slices.sh r06a 8 4
