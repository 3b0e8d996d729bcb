set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06r; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_dpll_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab.sh r06r 2 - "--workload uf250 --steps 4 --warmup 1;--workload 5sat-n200 --steps 4 --warmup 1;--workload uf250 --node-limit 0 --total 1024 --split-always --helpers-per-cu 16 --steps 2 --warmup 0" libsatmi_prev.so libsatmi.so || exit 1
PMC_GROUPS="sq1 sq2" bash tools/pmc_workload.sh r06r_uf uf250 "dpll_scan_kernel" --steps 2 --warmup 1 > /dev/null && echo uf sq ok
