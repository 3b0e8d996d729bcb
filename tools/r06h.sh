set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06h; mkdir -p $OUT
run() {  # name, bench args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$nm.json')); print('$nm', round(d['value'],2), round(d['ms_per_step']), round(d['wave_utilisation'],3), d['verdict_sha'], d['branch_split'])"
}
run uf_h10 --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu 10 --steps 2 --warmup 0
run uf_h16 --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu 16 --steps 2 --warmup 0
run uf_h24 --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu 24 --steps 2 --warmup 0
run uf1k_h16 --workload uf250 --node-limit 0 --total 1024 --split-always --helpers-per-cu 16 --steps 2 --warmup 0
run a12_4k_h1 --workload 5sat-n200-a12 --total 4096 --split-always --helpers-per-cu 1 --steps 2 --warmup 0
run a12_16k_h1 --workload 5sat-n200-a12 --total 16384 --split-always --helpers-per-cu 1 --steps 2 --warmup 0
