set -o pipefail
mkdir -p gpurun_out/dpab
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_driver_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dpab/tests.log 2>&1 || { tail -30 gpurun_out/dpab/tests.log; exit 1; }
tail -1 gpurun_out/dpab/tests.log
for i in 1 2 3; do
  for lib in libsatmi.so libsatmi_v.so; do
    SATMI_LIB_VARIANT=$lib timeout -k 10 200 python bench.py --workload php-dp --steps 20 --no-cpu-baseline > gpurun_out/dpab/${lib}_$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/dpab/${lib}_$i.json')); print('$lib', round(d['value'],2), round(d['ms_per_step'],2))"
  done
done
