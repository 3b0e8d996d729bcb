set -o pipefail
export TMPDIR=/tmp
EXTRA="--split-always" SUFFIX=_sa bash tools/slices.sh r06b 8 || exit 1
EXTRA="--split-always --helpers-per-cu 2" SUFFIX=_sa2 bash tools/slices.sh r06b 8 || exit 1
EXTRA="--split-always --split-warmup 64" SUFFIX=_saw64 bash tools/slices.sh r06b 8 || exit 1
timeout -k 10 200 python tools/fullsolve_probe.py 200 4223 5 5200 64 90 > gpurun_out/r06b/probe_5sat.jsonl 2> gpurun_out/r06b/probe_5sat.err || { tail -5 gpurun_out/r06b/probe_5sat.err; exit 1; }
tail -1 gpurun_out/r06b/probe_5sat.jsonl
