set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dpll_gpu.py tests/test_resolution_gpu.py -k "5sat200 or share_the_table" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for h in 1 4 10; do
  timeout -k 10 200 python bench.py --workload 5sat-n200-a12 --split-always --helpers-per-cu $h --steps 2 --warmup 1 --no-cpu-baseline --no-legs > $OUT/a12_h$h.json 2> $OUT/a12_h$h.err || { tail -5 $OUT/a12_h$h.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/a12_h$h.json')); print('h$h', d['value'], d['ms_per_step'], d['wave_utilisation'], d['capped_fraction'], d['resident_waves'])"
done
for v in "" dupcnt dupgather; do
  lib=${v:+libsatmi_$v.so}
  SATMI_LIB_VARIANT=${lib:-libsatmi.so} PMC_GROUPS="sq2" bash tools/pmc_workload.sh r06e_uf$v uf250 "dpll_scan_kernel" --steps 2 --warmup 1 > /dev/null || exit 1
  SATMI_LIB_VARIANT=${lib:-libsatmi.so} PMC_GROUPS="sq2" bash tools/pmc_workload.sh r06e_5s$v 5sat-n200 "dpll_scan_kernel" --steps 2 --warmup 1 > /dev/null || exit 1
  echo "variant ${v:-product}"; grep -E "LDS_IDX|BANK" gpurun_out/r06e_uf$v/pmc_uf250.txt gpurun_out/r06e_5s$v/pmc_5sat-n200.txt
done
