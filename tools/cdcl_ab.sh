# CDCL A/B on the GPU box: the CDCL GPU tests on the product library, then
# tools/cdcl_probe.py over variant libraries (VARIANTS, 2 reps) and phase builds (PHASES).
set -o pipefail
O=gpurun_out/${TAG:-cdclab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cdcl_gpu.py -x -q --timeout 240 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
for v in $VARIANTS; do
  SATMI_LIB_VARIANT=libsatmi_$v.so timeout -k 10 120 python tools/cdcl_probe.py --tag $v >> $O/ab.jsonl 2>>$O/ab.err || exit 1
done; done
for v in $PHASES; do
  SATMI_LIB_VARIANT=libsatmi_$v.so timeout -k 10 120 python tools/cdcl_probe.py --tag $v >> $O/phases.jsonl 2>>$O/ab.err || exit 1
done
cut -c1-100 $O/ab.jsonl; cat $O/phases.jsonl
