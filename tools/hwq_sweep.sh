set -o pipefail
for q in 4 17; do
  for t in 1 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --workload php-dp --steps 10 --warmup 2 --threads $t --no-cpu-baseline > gpurun_out/hwq_${q}_$t.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/hwq_${q}_$t.json').read().strip().splitlines()[-1]); print('queues $q threads $t', round(d['value'],1))"
  done
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --workload rand-dp --steps 3 --warmup 1 --threads 8 --no-cpu-baseline > gpurun_out/hwq_${q}_rdp.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/hwq_${q}_rdp.json').read().strip().splitlines()[-1]); print('queues $q rand-dp 8', round(d['value'],1))"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --workload cdcl --steps 3 --warmup 1 --threads 4 --no-cpu-baseline > gpurun_out/hwq_${q}_cdcl.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/hwq_${q}_cdcl.json').read().strip().splitlines()[-1]); print('queues $q cdcl 4', round(d['value'],1))"
done
