set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06n; mkdir -p $OUT
run() {  # name, bench args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$nm.json')); print('$nm', round(d['value'],2), round(d['ms_per_step']), round(d['wave_utilisation'],3), d['verdict_sha'], d['branch_split'])"
}
U="--workload uf250 --node-limit 0 --total 1024 --split-always --steps 2 --warmup 0"
run w64 $U --helpers-per-cu 16 --split-warmup 64
run w128 $U --helpers-per-cu 16 --split-warmup 128
run w512 $U --helpers-per-cu 16 --split-warmup 512
run h24 $U --helpers-per-cu 24
run h32 $U --helpers-per-cu 32
run s1 $U --helpers-per-cu 16 --streams 1
