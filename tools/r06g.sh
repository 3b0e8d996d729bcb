set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06g; mkdir -p $OUT
run() {  # name, bench args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$nm.json')); print('$nm', round(d['value'],2), round(d['ms_per_step']), round(d['wave_utilisation'],3), d['verdict_sha'], d['branch_split'])"
}
run uf_h16 --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu 16 --steps 2 --warmup 0
run uf_h24 --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu 24 --steps 2 --warmup 0
run uf_h16_w64 --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu 16 --split-warmup 64 --steps 2 --warmup 0
run uf_h16_w1k --workload uf250 --node-limit 0 --total 512 --split-always --helpers-per-cu 16 --split-warmup 1024 --steps 2 --warmup 0
run a12_8k_h1 --workload 5sat-n200-a12 --total 8192 --split-always --helpers-per-cu 1 --steps 2 --warmup 1
run a12_8k_h2 --workload 5sat-n200-a12 --total 8192 --split-always --helpers-per-cu 2 --steps 2 --warmup 1
run a12_2k_h1_w1k --workload 5sat-n200-a12 --total 2048 --split-always --helpers-per-cu 1 --split-warmup 1024 --steps 2 --warmup 1
