"""Summarise tools/pmc_req.sh's passes: per dispatch (in dispatch order) the
memory-side read requests by size and the bytes they carry.

usage: python tools/pmc_req_summarize.py <outdir>   -> <outdir>/pmc_req.json
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summarize import lib_sha16  # noqa: E402

KEYS = {"TCC_EA0_RDREQ_sum": "rdreq", "TCC_EA0_RDREQ_32B_sum": "rd32", "TCC_EA0_RDREQ_64B_sum": "rd64",
        "TCC_EA0_RDREQ_128B_sum": "rd128", "TCC_EA0_RDREQ_DRAM_sum": "rd_dram", "WRITE_SIZE": "write_kb"}


def per_dispatch(path, counter):
    v, names = {}, {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        d = int(r["Dispatch_Id"])
        v[d] = v.get(d, 0.0) + float(r["Counter_Value"])
        names[d] = r.get("Kernel_Name", "")[:100]
    ks = sorted(v)
    return [v[k] for k in ks], [names[k] for k in ks]


def main():
    out = sys.argv[1]
    cols, names = {}, None
    for c, k in KEYS.items():
        p = os.path.join(out, f"counters_{c}.csv")
        if os.path.exists(p):
            cols[k], nm = per_dispatch(p, c)
            names = names or nm
    n = min(len(x) for x in cols.values()) if cols else 0
    rows = []
    for i in range(n):
        r = {k: cols[k][i] for k in cols}
        r["kernel"] = names[i] if names and i < len(names) else ""
        if all(k in r for k in ("rd32", "rd64", "rd128")):
            r["read_bytes"] = 32 * r["rd32"] + 64 * r["rd64"] + 128 * r["rd128"]
            r["sized_reqs"] = r["rd32"] + r["rd64"] + r["rd128"]
        if "write_kb" in r:
            r["write_bytes"] = 1024 * r["write_kb"]
        rows.append(r)
    calib = sorted(glob.glob(os.path.join(out, "calib*.json")))
    res = {"lib_sha16": lib_sha16(), "dispatches": rows}
    if calib:
        c = json.load(open(calib[0]))["dispatches"]
        g = [r for r in rows if "k_gather" in r["kernel"]]
        res["calibration"] = [dict(e, **{k: x[k] for k in x if k != "kernel"},
                                   read_bytes_per_line=(x.get("read_bytes", 0) / e["lines"]),
                                   reqs_per_line=x.get("rdreq", 0) / e["lines"])
                              for e, x in zip(c, g[-len(c):])]
    json.dump(res, open(os.path.join(out, "pmc_req.json"), "w"), indent=1)
    print(json.dumps(res)[:3000])


if __name__ == "__main__":
    main()
