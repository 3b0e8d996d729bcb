set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06j; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o k -- python bench.py --workload php-dp --steps 5 --warmup 1 --no-cpu-baseline --no-legs > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/summary.txt && head -12 $OUT/summary.txt
