set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06k; mkdir -p $OUT
SATMI_DP_PHASES=1 timeout -k 10 100 python bench.py --workload php-dp --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
tail -4 $OUT/b.err
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 100 python bench.py --workload php-dp --steps 40 --warmup 3 --no-cpu-baseline --no-legs > $OUT/b40.json 2> $OUT/b40.err || exit 1
python -c "import json; d=json.load(open('$OUT/b40.json')); print('php-dp', d['value'], d['roofline']['launches_per_solve'], d['roofline']['device_ms_per_solve'])"
timeout -k 10 100 python bench.py --workload rand-dp --threads 8 --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $OUT/rd.json 2> $OUT/rd.err || exit 1
python -c "import json; d=json.load(open('$OUT/rd.json')); print('rand-dp 8 threads', d['value'])"
