#!/bin/bash
# Final SQ / HBM PMC passes of round 5 over the non-headline legs (tools/pmc_workload.sh), run through gpurun.
set -o pipefail
PMC_GROUPS="sq1 sq2" bash tools/pmc_workload.sh r05f_cdcl cdcl "cdcl_kernel" --steps 2 --warmup 1 && echo cdcl ok &&
PMC_GROUPS="sq1 sq2 fetch write" bash tools/pmc_workload.sh r05f_res php-res "res_pass" --steps 20 --warmup 3 && echo res ok &&
PMC_GROUPS="sq1 sq2" bash tools/pmc_workload.sh r05f_uf uf250 "dpll_scan_kernel" --steps 2 --warmup 1 && echo uf ok &&
PMC_GROUPS="sq1 sq2" bash tools/pmc_workload.sh r05f_5s 5sat-n200 "dpll_scan_kernel" --steps 2 --warmup 1 && echo 5sat ok
