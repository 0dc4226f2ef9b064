"""Per-dispatch durations of one kernel from a rocprofv3 --kernel-trace CSV.

usage: python tools/trace_durations.py <kernel_trace.csv> <kernel-name substring> [--last K] [--out f.json]
Prints (and writes) the durations in us in dispatch order, and their summary."""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernel")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    d = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            if args.kernel in r.get("Kernel_Name", ""):
                d.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                          r["Kernel_Name"][:120], int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)))
    d.sort()
    if args.last:
        d = d[-args.last:]
    us = [x[1] for x in d]
    grids = {}
    for x in d:   # by grid size (one launch shape each: e.g. the rank legs' 2^19 and 2^21 pairs)
        grids.setdefault(str(x[3]), []).append(x[1])
    res = {"kernel": args.kernel, "dispatches": len(us), "us": us,
           "by_grid": {g: {"dispatches": len(v), "us": v, "median_us": sorted(v)[len(v) // 2]} for g, v in grids.items()},
           "avg_us": sum(us) / len(us) if us else None, "min_us": min(us) if us else None,
           "max_us": max(us) if us else None, "names": sorted({x[2] for x in d})}
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
