#!/bin/bash
# Parity of the clause kernels (incl. the fused batch assignment) + split-auto A/B (run through gpurun).
set -o pipefail
OUT=gpurun_out/ab_auto
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_dpll_gpu.py tests/test_configs_gpu.py -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/gpu_tests.log | head; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for spec in "full:--steps 10" "share:--total 32768 --steps 20 --warmup 3" "share_ns:--total 32768 --steps 20 --warmup 3 --no-split" "n50:--workload 3sat-n50 --steps 20"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $OUT/$name.json 2>/dev/null || { echo "bench $name failed"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']), round(d['roofline']['kernel_ms'],1), d.get('branch_split'))"
done
