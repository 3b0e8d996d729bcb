set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06p; mkdir -p $OUT
SATMI_SPLIT_DEEP=1 timeout -k 10 600 python -u -m pytest tests/test_dpll_gpu.py -x -q --timeout 300 --timeout-method thread -k "splitting or solved_to_completion or bench_kernel" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() {  # name, bench args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$nm.json')); print('$nm', round(d['value'],2), round(d['ms_per_step']), d['wave_utilisation'], d['verdict_sha'])"
}
for deep in 0 1; do
  export SATMI_SPLIT_DEEP=$deep
  run uf_d$deep --workload uf250 --node-limit 0 --total 1024 --split-always --helpers-per-cu 16 --steps 2 --warmup 0
  run a12_d$deep --workload 5sat-n200-a12 --total 16384 --split-always --steps 2 --warmup 0
  run n8_d$deep --emulate-world 8 --emulate-rank 1 --steps 20 --warmup 5
done
