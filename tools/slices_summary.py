"""Summarise tools/slices.sh: per world size, every slice's rate and verdict
hash, and the imbalance factor mean / max of the per-slice step times (a
strong-scaling job's step time is the max over its ranks).

    python tools/slices_summary.py gpurun_out/<tag>/slices.jsonl <full-size bench line> > profiles/r06/slices.json
"""
import json
import sys


def main():
    rows = [json.loads(x) for x in open(sys.argv[1]) if x.strip()]
    full = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    out = {"full_size": {"value": full["value"], "ms_per_step": full["ms_per_step"],
                         "verdict_sha": full["verdict_sha"], "sat": full["last_step_totals"]["sat"]},
           "worlds": {}}
    for N in sorted({r["world"] for r in rows}):
        sl = sorted((r for r in rows if r["world"] == N), key=lambda r: r["rank"])
        ms = [r["ms_per_step"] for r in sl]
        mean, mx = sum(ms) / len(ms), max(ms)
        total = sum(r["shard"]["end"] - r["shard"]["begin"] for r in sl)
        job_rate = total / (mx * 1e-3)   # every rank at its own slice's rate, the job at the slowest
        out["worlds"][str(N)] = {
            "slices": sl, "imbalance_mean_over_max": mean / mx,
            "slowest_rank": max(sl, key=lambda r: r["ms_per_step"])["rank"],
            "share_mean": sum(r["value"] for r in sl) / len(sl) / full["value"],
            "share_slowest": min(r["value"] for r in sl) / full["value"],
            "job_rate_bound": N * total / N / (mx * 1e-3),
            "job_efficiency_bound": job_rate / (N * full["value"]),
            "sat_sum": sum(r["sat"] for r in sl), "sat_full": full["last_step_totals"]["sat"],
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
