"""Wall time of one resolve() call on the php-res bench workload (PHP(4,3),
first 4 passes): median of 50 calls; [lib tag] in argv (SATMI_LIB_VARIANT picks
the library).  A/B helper for the host side of csrc/resolution.hip."""
import sys, time, json
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sat-mpi-stana-andrei_amd'))
import numpy as np
from satmi import cnf
from satmi.resolution import resolve, last_stats
f = cnf.pigeonhole(3)
for _ in range(3): resolve(f, max_passes=4)
ts = []
for _ in range(50):
    t = time.perf_counter(); r = resolve(f, max_passes=4); ts.append(time.perf_counter() - t)
st = last_stats()
print(json.dumps({"lib": sys.argv[1] if len(sys.argv) > 1 else "", "median_ms": float(np.median(ts)) * 1e3, "min_ms": min(ts) * 1e3,
                  "pair_ms": st["pair_ms"], "pass_new": r["pass_new"], "derived_per_s": sum(r["pass_new"]) / float(np.median(ts))}))
