#!/bin/bash
# SQ passes over the configs[4] legs (uf250, 5-SAT n=200) at their bench sizes, one
# directory per workload (tools/pmc_workload.sh), then the default bench line.
# Usage (through gpurun): bash tools/pmc_c4.sh <tag>
set -o pipefail
TAG=${1:-c4}
PMC_GROUPS="sq1 sq2" bash tools/pmc_workload.sh ${TAG}_uf uf250 "dpll_scan_kernel" --steps 2 --warmup 1 && echo uf ok &&
PMC_GROUPS="sq1 sq2" bash tools/pmc_workload.sh ${TAG}_5s 5sat-n200 "dpll_scan_kernel" --steps 2 --warmup 1 && echo 5sat ok
