"""Wall time of one resolve() call on the php-res bench workload (PHP(4,3),
first 4 passes): median of 50 calls; [lib tag] in argv (SATMI_LIB_VARIANT picks
the library).  A/B helper for the host side of csrc/resolution.hip.  Beside it:
the C call alone (satmi_resolution_host on prebuilt arrays: the Python
wrapper's share is the difference), the pass kernels' device time and their
live shader clock."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sat-mpi-stana-andrei_amd'))
if "--torch" in sys.argv:   # as bench.py: torch (and its HIP runtime setup) loaded first
    import torch  # noqa: F401,E402
    torch.cuda.set_device(0)
import numpy as np  # noqa: E402
from satmi import _capi, cnf  # noqa: E402
from satmi.resolution import _csr, _p, last_stats, resolve  # noqa: E402

f = cnf.pigeonhole(3)
for _ in range(3):
    resolve(f, max_passes=4)
ts = []
for _ in range(50):
    t = time.perf_counter()
    r = resolve(f, max_passes=4)
    ts.append(time.perf_counter() - t)
st = last_stats()
L = _capi.load()
off, lits = _csr(f)
res, passes = ctypes.c_int32(0), ctypes.c_int32(0)
pn = np.zeros(4, dtype=np.int64)
tc = []
for _ in range(50):
    t = time.perf_counter()
    L.satmi_resolution_host(len(f), _p(off), _p(lits), 4, 0, 0.0, ctypes.byref(res), ctypes.byref(passes),
                            _p(pn, ctypes.c_int64), 4, None, 0, None, 0, None, 0)
    tc.append(time.perf_counter() - t)
print(json.dumps({"lib": " ".join(sys.argv[1:]), "median_ms": float(np.median(ts)) * 1e3,
                  "min_ms": min(ts) * 1e3, "c_call_median_ms": float(np.median(tc)) * 1e3,
                  "pair_ms": st["pair_ms"], "shader_clock_hz": st.get("shader_clock_hz"), "pass_new": r["pass_new"],
                  "derived_per_s": sum(r["pass_new"]) / float(np.median(ts))}))
