set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06q; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_dpll_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab.sh r06q 2 - "--workload uf250 --total 7680 --steps 4 --warmup 1;--workload uf250 --total 8192 --steps 4 --warmup 1;--workload 5sat-n200 --steps 4 --warmup 1" libsatmi_prev.so libsatmi.so
