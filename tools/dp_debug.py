"""Debug aid: one Davis-Putnam formula on the GPU next to the oracle (record mode and not)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sat-mpi-stana-andrei_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from satmi.dp import eliminate  # noqa: E402

fs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [[[-10, 5, 2], [-2], [-6, 2], [1, -1, 2], [-10, 5, 2]]]
for f in fs:
    o = oracle.dp(f, record=True)
    r = eliminate(f, record=True)
    r2 = eliminate(f)
    print("formula", f)
    print(" oracle", o["result"], o["vars"], o["clauses"])
    print(" gpu   ", r["result"], r["vars"], r["clauses"])
    print(" gpu2  ", r2["result"], r2["vars"])
