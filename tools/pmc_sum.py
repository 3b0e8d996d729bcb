"""Sum rocprofv3 --output-format csv counter rows per (kernel, counter).

    python tools/pmc_sum.py gpurun_out/pmc2/pmc2_counter_collection.csv [kernel-substring]
"""
import collections
import csv
import sys


def summarize(path, kfilter="dpll"):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if kfilter not in row.get("Kernel_Name", ""):
                continue
            agg[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row.get("Dispatch_Id"))
    return {k: (v, len(disp[k])) for k, v in sorted(agg.items())}


if __name__ == "__main__":
    for k, (v, nd) in summarize(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "dpll").items():
        print(f"{k:28s} {v:18.0f}  dispatches={nd}")
