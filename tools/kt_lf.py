"""Per-dispatch durations of the LF kernels from a rocprofv3 kernel trace, beside
the event times tools/rank_queued.py measured in the same run.

rank_queued times each (variant, size) as graph replays (cold, ptewarm, warm)
and, with --eager, as direct launches (cold, warm), reps launches each, after
one capture warm-up launch; the trace lists the dispatches in that order, so the
k-th LF dispatch of a grid size is matched to its timed launch by position.
usage: python tools/kt_lf.py <kernel_trace.csv> <rq.json> [--out file.json]
"""
import argparse
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("rq")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if "k_lf" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    disp = [{"kernel": r["Kernel_Name"].split("(")[0].split("::")[-1].replace("void ", ""),
             "grid": int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0),
             "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3} for r in rows]
    rq = json.load(open(args.rq))
    # group consecutive dispatches by grid size into runs; the timed launches of one
    # (variant, size) entry are the last 5 * (3 + 2) dispatches of its run
    runs = []
    for d in disp:
        if runs and runs[-1]["grid"] == d["grid"] and runs[-1]["kernel"] == d["kernel"]:
            runs[-1]["us"].append(d["us"])
        else:
            runs.append({"kernel": d["kernel"], "grid": d["grid"], "us": [d["us"]]})
    out = {"runs": [], "entries": []}
    for r in runs:
        out["runs"].append({"kernel": r["kernel"], "grid": r["grid"], "n": len(r["us"]),
                            "us": [round(x, 2) for x in r["us"]]})
    ents = [e for e in rq.get("rank", []) if "error" not in e]
    # (offset within the entry's last 35 dispatches, stride) of each temperature's timed launches
    temps = {"cold": (0, 1), "ptewarm": (5, 1), "warm": (11, 2), "eager_cold": (20, 1), "eager_warm": (26, 2)}
    big = [r for r in runs if len(r["us"]) >= 35]
    for e, r in zip(ents, big):
        k = len(r["us"]) - 35
        res = {"lf_work": e["lf_work"], "pairs_log2": e["pairs_log2"], "kernel": r["kernel"], "grid": r["grid"]}
        for t, (o, st) in temps.items():
            ker = r["us"][k + o: k + o + 5 * st: st]
            res[t + "_event_median_us"] = e.get(t + "_median_us")
            res[t + "_kernel_median_us"] = float(np.median(ker))
        out["entries"].append(res)
        print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
