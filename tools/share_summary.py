"""Collect share-sweep bench lines (tools/share_sweep.sh / ad-hoc --total runs)
into one JSON: per run the arguments, instances/s, ms/step, verdict hash, and
the ratio to the full-size (262,144 per step) line of the same box.

    python tools/share_summary.py <out.json> <dir>...
"""
import glob
import json
import os
import sys


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    runs = []
    for d in dirs:
        for f in sorted(glob.glob(os.path.join(d, "*.json"))):
            try:
                line = json.loads(open(f).read().strip().splitlines()[-1])
            except (ValueError, IndexError):
                continue
            c = line.get("config", {})
            runs.append({"file": os.path.relpath(f), "box": d, "instances_per_step": c.get("instances_per_step"),
                         "streams": c.get("streams"), "value": line["value"], "ms_per_step": line["ms_per_step"],
                         "steps": line["steps"], "verdict_sha": line.get("verdict_sha"),
                         "split_launch": bool(line.get("branch_split")),
                         "split_policy": c.get("split_policy", "auto" if c.get("branch_splitting") else "off"),
                         "helpers_per_cu": c.get("helpers_per_cu"), "split_warmup": c.get("split_warmup")})
    for d in dirs:
        full = [r["value"] for r in runs if r["box"] == d and r["instances_per_step"] == 262144]
        ref = sum(full) / len(full) if full else None
        for r in runs:
            if r["box"] == d and ref:
                r["ratio_to_full_same_box"] = r["value"] / ref
    json.dump({"runs": runs}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
