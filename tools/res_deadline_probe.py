"""The resolution deadline on a saturation far beyond it: PHP(5,4) (its 5th
pass resolves ~10^16 pairs) with time limits of 0.3 s and 1 s, three calls in
one process (the first grows the workspace).  Prints each call's wall time,
verdict (-1 = stopped by the limit) and completed passes."""
import sys, time, json
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, 'sat-mpi-stana-andrei_amd'), os.path.join(_R, 'oracle')]
from satmi import cnf
from satmi.resolution import resolve, last_stats
f = cnf.pigeonhole(4)
for tl in (0.3, 0.3, 1.0):
    t = time.perf_counter(); r = resolve(f, time_limit=tl); dt = time.perf_counter() - t
    print(json.dumps({"lib": sys.argv[1], "tl": tl, "dt": dt, "result": r["result"], "passes": r["passes"], "pass_new": r["pass_new"]}), flush=True)
