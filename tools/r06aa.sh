# SQ instruction mix of the headline launch: unsplit (default) vs split form (--split-always), one launch each
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06aa; mkdir -p $OUT
for v in "def:" "split:--split-always"; do
  n=${v%%:*}; a=${v#*:}
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
    --output-format csv -d "$PWD/$OUT/$n" -o p -- python bench.py --steps 1 --warmup 0 --profile-steps --no-legs $a > $OUT/$n.json 2> $OUT/$n.err || exit 1
  python tools/pmc_sum.py "$(find $OUT/$n -name '*counter_collection.csv' | head -1)" dpll_fixed_kernel > $OUT/$n.txt
  rm -rf $OUT/$n
  echo "== $n"; cat $OUT/$n.txt
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('nodes', d['last_step_totals'])"
done
