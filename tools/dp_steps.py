"""Per-step kernel durations of the last PHP(6,5) solve in a rocprofv3 kernel
trace of tools/dp_trace_probe.py (us per kernel, per elimination step).

    python tools/dp_steps.py gpurun_out/<tag>/kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "pop_split" in r["Kernel_Name"]]
    last = idx[-30:]
    tot = {}
    span = 0.0
    for a, b in zip(last, last[1:] + [len(rows)]):
        ks = [k for k in rows[a:b] if "rocclr" not in k["Kernel_Name"]]
        d = {}
        for k in ks:
            n = k["Kernel_Name"].split("(")[0].replace("satmi::", "").replace("void ", "")
            n = n.replace("dp_", "").replace("_kernel", "")
            us = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1000
            d[n] = d.get(n, 0) + us
            tot[n] = tot.get(n, 0) + us
        s = (int(ks[-1]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"])) / 1000
        span += s
        print(f"{s:7.1f}us " + " ".join(f"{n}:{v:.1f}" for n, v in d.items()))
    print(f"span {span:.1f} us; per kernel: " + " ".join(f"{n}:{v:.0f}" for n, v in tot.items()))


if __name__ == "__main__":
    main(sys.argv[1])
