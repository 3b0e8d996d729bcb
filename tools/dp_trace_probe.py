"""One PHP(6,5) Davis-Putnam solve after warm-up, for a kernel trace
(rocprofv3 --kernel-trace): per-step kernel durations of the device pipeline."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sat-mpi-stana-andrei_amd"))
from satmi import cnf  # noqa: E402
from satmi.dp import eliminate  # noqa: E402

f = cnf.pigeonhole(5)
for _ in range(3):
    r = eliminate(f)
print(r["result"], r["steps"])
