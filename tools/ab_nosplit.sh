set -o pipefail
mkdir -p gpurun_out/ab_ns
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab_ns/split_$i.json 2>/dev/null || exit 1
  SATMI_LIB_VARIANT=libsatmi_nosplit.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --no-split > gpurun_out/ab_ns/nosplit_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/ab_ns/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), round(d['roofline']['kernel_ms'],1))"; done
