"""Summarise a rocprofv3 kernel-trace database (results.db): per-kernel totals,
and the dispatch timeline of the last `--last N` dispatches."""
import argparse
import glob
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("path")
ap.add_argument("--last", type=int, default=0)
a = ap.parse_args()
db = a.path if a.path.endswith(".db") else sorted(glob.glob(a.path + "/**/*.db", recursive=True))[-1]
c = sqlite3.connect(db)
for r in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels limit 25"):
    print(f"{r[0][:60]:60s} calls {r[1]:6d} total {r[2] / 1e3:9.3f} ms avg {r[3]:9.2f} us {r[4]:5.1f}%")
if a.last:
    rows = list(c.execute("select name,start,end,grid_x,grid_y from kernels order by start"))[-a.last:]
    prev = rows[0][1]
    for n, s, e, gx, gy in rows:
        print(f"{n.split('(')[0][-34:]:34s} dur {(e - s) / 1e3:8.1f} us gap {(s - prev) / 1e3:6.1f} us grid {gx}x{gy}")
        prev = e
    print("span us", (rows[-1][2] - rows[0][1]) / 1e3)
