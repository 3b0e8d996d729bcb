#!/bin/bash
# configs[4] solved-to-the-end leg: batch size / steps / helper waves per CU sweep (through gpurun).
# Usage: bash tools/solved_sweep.sh "<cfg>;<cfg>..."   (default: the batch / steps sweep)
set -o pipefail
mkdir -p gpurun_out/solved
CFGS=${1:-"--total 512 --steps 2;--total 512 --steps 4;--total 1024 --steps 2"}
IFS=';' read -r -a LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  f=gpurun_out/solved/$(echo $cfg | tr -d ' -').json
  timeout -k 10 300 python bench.py --workload uf250 --node-limit 0 --split-always --warmup 0 --no-cpu-baseline --no-legs $cfg > $f 2> ${f%.json}.err || exit 1
  python -c "import json; d=json.load(open('$f')); print('$cfg', round(d['value'],2), round(d['ms_per_step']), round(d['wave_utilisation'],3), d['verdict_sha'])"
done
